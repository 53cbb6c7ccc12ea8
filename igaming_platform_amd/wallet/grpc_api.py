"""wallet.v1 gRPC server and client (services/wallet/cmd/main.go:66-311).

Errors map to gRPC status codes; the wallet error code (wallet.proto:233-241) travels in the
``wallet-error-code`` trailing metadata and the status details string. The wallet logs every
request at info (main.go:281-285), unlike risk.
"""
from __future__ import annotations

import time
from concurrent import futures
from typing import Optional

import grpc

from ..api.grpc_server import HealthServicer, MetricsInterceptor, RecoveryInterceptor, health_handler
from ..obs.logging import get_logger
from ..obs.metrics import Metrics
from ..proto import wallet_v1 as W
from .domain import WalletError
from .service import WalletService

log = get_logger("wallet.grpc")

STATUS = {
    "ACCOUNT_NOT_FOUND": grpc.StatusCode.NOT_FOUND, "TRANSACTION_NOT_FOUND": grpc.StatusCode.NOT_FOUND,
    "INSUFFICIENT_BALANCE": grpc.StatusCode.FAILED_PRECONDITION,
    "ACCOUNT_SUSPENDED": grpc.StatusCode.FAILED_PRECONDITION,
    "BONUS_RESTRICTION": grpc.StatusCode.FAILED_PRECONDITION,
    "INVALID_OPERATION": grpc.StatusCode.FAILED_PRECONDITION,
    "DUPLICATE_TRANSACTION": grpc.StatusCode.ALREADY_EXISTS, "DUPLICATE_ACCOUNT": grpc.StatusCode.ALREADY_EXISTS,
    "RISK_BLOCKED": grpc.StatusCode.PERMISSION_DENIED, "RISK_REVIEW": grpc.StatusCode.ABORTED,
    "INVALID_AMOUNT": grpc.StatusCode.INVALID_ARGUMENT, "INVALID_ARGUMENT": grpc.StatusCode.INVALID_ARGUMENT,
    "CONCURRENT_UPDATE": grpc.StatusCode.ABORTED,
}


def _ts(sec: Optional[float]):
    t = W.Timestamp()
    if sec:
        t.seconds = int(sec)
        t.nanos = int((sec - int(sec)) * 1e9)
    return t


def tx_pb(t):
    return W.Transaction(id=t.id, account_id=t.account_id, idempotency_key=t.idempotency_key, type=t.type,
                         amount=t.amount, balance_before=t.balance_before, balance_after=t.balance_after,
                         status=t.status, reference=t.reference, game_id=t.game_id or "", round_id=t.round_id or "",
                         risk_score=t.risk_score or 0, created_at=_ts(t.created_at),
                         completed_at=_ts(t.completed_at) if t.completed_at else None)


def acct_pb(a):
    return W.Account(id=a.id, player_id=a.player_id, currency=a.currency, balance=a.balance, bonus=a.bonus,
                     status=a.status, created_at=_ts(a.created_at), updated_at=_ts(a.updated_at))


class WalletServicer:
    def __init__(self, svc: WalletService):
        self.s = svc

    def CreateAccount(self, r, ctx):
        return W.CreateAccountResponse(account=acct_pb(self.s.create_account(r.player_id, r.currency)))

    def GetAccount(self, r, ctx):
        return W.GetAccountResponse(account=acct_pb(self.s.get_account(r.account_id, r.player_id)))

    def GetBalance(self, r, ctx):
        a = self.s.get_balance(r.account_id)
        return W.GetBalanceResponse(account_id=a.id, balance=a.balance, bonus=a.bonus, total=a.total_balance(),
                                    withdrawable=a.withdrawable(), currency=a.currency)

    def Deposit(self, r, ctx):
        t, nb, score = self.s.deposit(r.account_id, r.amount, r.idempotency_key, r.payment_method, r.reference,
                                      r.ip_address, r.device_id, r.fingerprint)
        return W.DepositResponse(transaction=tx_pb(t), new_balance=nb, risk_score=score or 0)

    def Withdraw(self, r, ctx):
        t, nb, score, st = self.s.withdraw(r.account_id, r.amount, r.idempotency_key, r.payout_method,
                                           r.payout_details, r.ip_address, r.device_id)
        return W.WithdrawResponse(transaction=tx_pb(t), new_balance=nb, risk_score=score or 0, payout_status=st)

    def Bet(self, r, ctx):
        t, nb, score, real, bonus = self.s.bet(r.account_id, r.amount, r.idempotency_key, r.game_id, r.round_id,
                                               r.game_category, r.ip_address, r.device_id, r.session_id)
        return W.BetResponse(transaction=tx_pb(t), new_balance=nb, risk_score=score or 0, real_deducted=real,
                             bonus_deducted=bonus)

    def Win(self, r, ctx):
        t, nb = self.s.win(r.account_id, r.amount, r.idempotency_key, r.game_id, r.round_id, r.bet_transaction_id,
                           r.win_type or "normal", dict(r.metadata))
        return W.WinResponse(transaction=tx_pb(t), new_balance=nb)

    def Refund(self, r, ctx):
        t, nb = self.s.refund(r.account_id, r.original_transaction_id, r.idempotency_key, r.reason)
        return W.RefundResponse(transaction=tx_pb(t), new_balance=nb)

    def GetTransactionHistory(self, r, ctx):
        t_from = r.__getattribute__("from").seconds if r.HasField("from") else None
        t_to = r.to.seconds if r.HasField("to") else None
        txs, total, more = self.s.history(r.account_id, r.limit or 50, r.offset, list(r.types), t_from, t_to,
                                          r.game_id)
        return W.GetTransactionHistoryResponse(transactions=[tx_pb(t) for t in txs], total=total, has_more=more)

    def GetTransaction(self, r, ctx):
        return W.GetTransactionResponse(transaction=tx_pb(self.s.get_transaction(r.transaction_id)))


def _errors(fn):
    def call(req, ctx):
        t0 = time.perf_counter()
        try:
            return fn(req, ctx)
        except WalletError as e:
            ctx.set_trailing_metadata((("wallet-error-code", e.code),))
            ctx.abort(STATUS.get(e.code, grpc.StatusCode.UNKNOWN), f"{e.code}: {e.message}")
        finally:
            log.info("wallet request", extra={"fields": dict(method=fn.__name__,
                                                             duration_ms=round((time.perf_counter() - t0) * 1e3, 3))})
    return call


def wallet_handler(servicer: WalletServicer) -> grpc.GenericRpcHandler:
    ser = lambda m: m.SerializeToString()  # noqa: E731
    return grpc.method_handlers_generic_handler(W.SERVICE, {
        rpc: grpc.unary_unary_rpc_method_handler(_errors(getattr(servicer, rpc)),
                                                 request_deserializer=W.M[req].FromString, response_serializer=ser)
        for rpc, req, _ in W.METHODS})


class WalletServer:
    def __init__(self, svc: WalletService, port: int = 0, host: str = "127.0.0.1", workers: int = 32):
        self.metrics = Metrics()
        self.health = HealthServicer()
        self.health.set(W.SERVICE, "SERVING")
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                                  interceptors=[RecoveryInterceptor(), MetricsInterceptor(self.metrics)])
        self.server.add_generic_rpc_handlers([wallet_handler(WalletServicer(svc)), health_handler(self.health)])
        self.port = self.server.add_insecure_port(f"{host}:{port}")

    def start(self) -> "WalletServer":
        self.server.start()
        return self

    def stop(self, grace: float = 1.0) -> None:
        self.health.set("", "NOT_SERVING")
        self.server.stop(grace).wait()


class WalletClient:
    def __init__(self, target: str, timeout_s: float = 5.0):
        self.channel = grpc.insecure_channel(target)
        self.timeout = timeout_s
        ser = lambda m: m.SerializeToString()  # noqa: E731
        self._m = {rpc: self.channel.unary_unary(W.method_path(rpc), request_serializer=ser,
                                                 response_deserializer=W.M[resp].FromString)
                   for rpc, _, resp in W.METHODS}

    def call(self, rpc: str, **kw):
        req_type = next(r for n, r, _ in W.METHODS if n == rpc)
        return self._m[rpc](W.M[req_type](**kw), timeout=self.timeout)

    def close(self) -> None:
        self.channel.close()
