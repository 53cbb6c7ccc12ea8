"""risk.v1 gRPC client (the ``RiskService`` the wallet/bonus services consume:
wallet_service.go:40-42, 123-138; bonus_engine.go:139-141)."""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import grpc

from ..proto import health_v1 as HV
from ..proto import risk_v1 as P


class RiskClient:
    def __init__(self, target: str, timeout_s: float = 5.0, channel: Optional[grpc.Channel] = None):
        self.channel = channel or grpc.insecure_channel(target, options=[("grpc.max_receive_message_length", 64 << 20),
                                                                          ("grpc.max_send_message_length", 64 << 20)])
        self.timeout = timeout_s
        ser = lambda m: m.SerializeToString()  # noqa: E731
        self._m = {}
        for rpc, req, resp in P.METHODS:
            self._m[rpc] = self.channel.unary_unary(P.method_path(rpc), request_serializer=ser,
                                                    response_deserializer=P.M[resp].FromString)
        self._raw_batch = self.channel.unary_unary(P.method_path("ScoreBatch"))
        self._health = self.channel.unary_unary(f"/{HV.SERVICE}/Check", request_serializer=ser,
                                                response_deserializer=HV.HealthCheckResponse.FromString)

    def close(self) -> None:
        self.channel.close()

    def call(self, rpc: str, req, timeout: Optional[float] = None):
        return self._m[rpc](req, timeout=timeout or self.timeout)

    # ---- convenience wrappers
    def score(self, account_id: str, amount: int, transaction_type: str, **kw):
        return self.call("ScoreTransaction", P.ScoreTransactionRequest(account_id=account_id, amount=amount,
                                                                       transaction_type=transaction_type, **kw))

    def score_batch(self, txs: Sequence[Dict]):
        req = P.ScoreBatchRequest(transactions=[P.ScoreTransactionRequest(**t) for t in txs])
        return self.call("ScoreBatch", req)

    def score_batch_raw(self, payload: bytes, timeout: Optional[float] = None) -> bytes:
        return self._raw_batch(payload, timeout=timeout or self.timeout)

    def predict_ltv(self, account_id: str):
        return self.call("PredictLTV", P.PredictLTVRequest(account_id=account_id))

    def player_segment(self, account_id: str):
        return self.call("GetPlayerSegment", P.GetPlayerSegmentRequest(account_id=account_id))

    def check_bonus_abuse(self, account_id: str, bonus_id: str = ""):
        return self.call("CheckBonusAbuse", P.CheckBonusAbuseRequest(account_id=account_id, bonus_id=bonus_id))

    def add_to_blacklist(self, type_: str, value: str, reason: str = "", created_by: str = "", expires_at: int = 0):
        req = P.AddToBlacklistRequest(type=type_, value=value, reason=reason, created_by=created_by)
        if expires_at:
            req.expires_at.seconds = int(expires_at)
        return self.call("AddToBlacklist", req)

    def check_blacklist(self, device_id: str = "", fingerprint: str = "", ip_address: str = "", email: str = ""):
        return self.call("CheckBlacklist", P.CheckBlacklistRequest(device_id=device_id, fingerprint=fingerprint,
                                                                   ip_address=ip_address, email=email))

    def get_features(self, account_id: str):
        return self.call("GetFeatures", P.GetFeaturesRequest(account_id=account_id))

    def update_thresholds(self, block: int, review: int):
        return self.call("UpdateThresholds", P.UpdateThresholdsRequest(block_threshold=block, review_threshold=review))

    def get_thresholds(self):
        return self.call("GetThresholds", P.GetThresholdsRequest())

    def health(self, service: str = "") -> str:
        r = self._health(HV.HealthCheckRequest(service=service), timeout=self.timeout)
        return {v: k for k, v in HV.STATUS.items()}[r.status]
