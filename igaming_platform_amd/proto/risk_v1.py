"""``risk.v1`` wire contract, built in code (field numbers from proto/risk/v1/risk.proto).

Package, service and method names are identical to the reference
(``/root/reference/proto/risk/v1/risk.proto:1-32``) so existing clients and grpcurl
invocations (``Makefile:231-241``) work unchanged. Full method path:
``/risk.v1.RiskService/<Rpc>``.
"""
from __future__ import annotations

from .builder import build_file, enum_values, timestamp_class

FILE = "risk/v1/risk.proto"
PACKAGE = "risk.v1"
SERVICE = "risk.v1.RiskService"
TS = ".google.protobuf.Timestamp"

ENUMS = {
    "Action": [("ACTION_UNSPECIFIED", 0), ("ACTION_APPROVE", 1), ("ACTION_REVIEW", 2),
               ("ACTION_BLOCK", 3)],
    "Segment": [("SEGMENT_UNSPECIFIED", 0), ("SEGMENT_VIP", 1), ("SEGMENT_HIGH", 2),
                ("SEGMENT_MEDIUM", 3), ("SEGMENT_LOW", 4), ("SEGMENT_CHURNING", 5)],
}

MESSAGES = {
    "ScoreTransactionRequest": [
        ("account_id", 1, "string"), ("player_id", 2, "string"), ("amount", 3, "int64"),
        ("transaction_type", 4, "string"), ("currency", 5, "string"), ("game_id", 6, "string"),
        ("round_id", 7, "string"), ("ip_address", 8, "string"), ("device_id", 9, "string"),
        ("fingerprint", 10, "string"), ("user_agent", 11, "string"), ("session_id", 12, "string"),
        ("metadata", 13, None, "map:string:string"),
    ],
    "ScoreTransactionResponse": [
        ("score", 1, "int32"), ("action", 2, "enum:.risk.v1.Action"),
        ("reason_codes", 3, "string", "rep"), ("rule_score", 4, "int32"),
        ("ml_score", 5, "float"), ("response_time_ms", 6, "int64"),
        ("features", 7, ".risk.v1.FeatureVector"),
    ],
    "ScoreBatchRequest": [("transactions", 1, ".risk.v1.ScoreTransactionRequest", "rep")],
    "ScoreBatchResponse": [("results", 1, ".risk.v1.ScoreTransactionResponse", "rep")],
    "PredictLTVRequest": [("account_id", 1, "string")],
    "PredictLTVResponse": [
        ("account_id", 1, "string"), ("predicted_ltv", 2, "float"),
        ("segment", 3, "enum:.risk.v1.Segment"), ("churn_risk", 4, "float"),
        ("predicted_active_days", 5, "int32"), ("confidence", 6, "float"),
        ("next_best_action", 7, "string"), ("predicted_at", 8, TS),
    ],
    "GetPlayerSegmentRequest": [("account_id", 1, "string")],
    "GetPlayerSegmentResponse": [
        ("account_id", 1, "string"), ("segment", 2, "enum:.risk.v1.Segment"),
        ("ltv", 3, "float"), ("churn_risk", 4, "float"),
        ("recommended_actions", 5, "string", "rep"),
    ],
    "CheckBonusAbuseRequest": [("account_id", 1, "string"), ("bonus_id", 2, "string")],
    "CheckBonusAbuseResponse": [
        ("is_abuser", 1, "bool"), ("abuse_score", 2, "float"), ("signals", 3, "string", "rep"),
        ("linked_accounts", 4, "string", "rep"),
    ],
    "AddToBlacklistRequest": [
        ("type", 1, "string"), ("value", 2, "string"), ("reason", 3, "string"),
        ("created_by", 4, "string"), ("expires_at", 5, TS),
    ],
    "AddToBlacklistResponse": [("success", 1, "bool"), ("id", 2, "string")],
    "CheckBlacklistRequest": [
        ("device_id", 1, "string"), ("fingerprint", 2, "string"), ("ip_address", 3, "string"),
        ("email", 4, "string"),
    ],
    "CheckBlacklistResponse": [
        ("is_blacklisted", 1, "bool"), ("matches", 2, ".risk.v1.BlacklistMatch", "rep"),
    ],
    "BlacklistMatch": [
        ("type", 1, "string"), ("value", 2, "string"), ("reason", 3, "string"),
        ("created_at", 4, TS),
    ],
    "GetFeaturesRequest": [("account_id", 1, "string")],
    "GetFeaturesResponse": [
        ("account_id", 1, "string"), ("features", 2, ".risk.v1.FeatureVector"),
        ("computed_at", 3, TS),
    ],
    "FeatureVector": [
        ("tx_count_1m", 1, "int32"), ("tx_count_5m", 2, "int32"), ("tx_count_1h", 3, "int32"),
        ("tx_sum_1h", 4, "int64"), ("tx_avg_1h", 5, "float"), ("unique_devices_24h", 6, "int32"),
        ("unique_ips_24h", 7, "int32"), ("ip_country_changes_7d", 8, "int32"),
        ("device_age_days", 9, "int32"), ("account_age_days", 10, "int32"),
        ("total_deposits", 11, "int64"), ("total_withdrawals", 12, "int64"),
        ("net_deposit", 13, "int64"), ("deposit_count", 14, "int32"),
        ("withdraw_count", 15, "int32"), ("time_since_last_tx_sec", 16, "int32"),
        ("session_duration_sec", 17, "int32"), ("avg_bet_size", 18, "float"),
        ("win_rate", 19, "float"), ("is_vpn", 20, "bool"), ("is_proxy", 21, "bool"),
        ("is_tor", 22, "bool"), ("disposable_email", 23, "bool"),
        ("bonus_claim_count", 24, "int32"), ("bonus_wager_completion_rate", 25, "float"),
        ("bonus_only_player", 26, "bool"),
    ],
    "UpdateThresholdsRequest": [("block_threshold", 1, "int32"), ("review_threshold", 2, "int32")],
    "UpdateThresholdsResponse": [
        ("success", 1, "bool"), ("block_threshold", 2, "int32"), ("review_threshold", 3, "int32"),
    ],
    "GetThresholdsRequest": [],
    "GetThresholdsResponse": [("block_threshold", 1, "int32"), ("review_threshold", 2, "int32")],
}

# rpc name -> (request message, response message); order as in risk.proto:10-32
METHODS = [
    ("ScoreTransaction", "ScoreTransactionRequest", "ScoreTransactionResponse"),
    ("ScoreBatch", "ScoreBatchRequest", "ScoreBatchResponse"),
    ("PredictLTV", "PredictLTVRequest", "PredictLTVResponse"),
    ("GetPlayerSegment", "GetPlayerSegmentRequest", "GetPlayerSegmentResponse"),
    ("CheckBonusAbuse", "CheckBonusAbuseRequest", "CheckBonusAbuseResponse"),
    ("AddToBlacklist", "AddToBlacklistRequest", "AddToBlacklistResponse"),
    ("CheckBlacklist", "CheckBlacklistRequest", "CheckBlacklistResponse"),
    ("GetFeatures", "GetFeaturesRequest", "GetFeaturesResponse"),
    ("UpdateThresholds", "UpdateThresholdsRequest", "UpdateThresholdsResponse"),
    ("GetThresholds", "GetThresholdsRequest", "GetThresholdsResponse"),
]

# map field needs no scalar type in the spec tuple; patch it for the builder
MESSAGES["ScoreTransactionRequest"][-1] = ("metadata", 13, "string", "map:string:string")

M = build_file(FILE, PACKAGE, MESSAGES, ENUMS,
               services={"RiskService": METHODS}, deps=["google/protobuf/timestamp.proto"])
Timestamp = timestamp_class()
ACTION = enum_values("risk.v1.Action")
SEGMENT = enum_values("risk.v1.Segment")


def method_path(rpc: str) -> str:
    return f"/{SERVICE}/{rpc}"


def __getattr__(name):
    if name in M:
        return M[name]
    raise AttributeError(name)
