"""``wallet.v1`` wire contract built in code (field numbers of proto/wallet/v1/wallet.proto).

Service ``wallet.v1.WalletService`` with the reference's 10 RPCs (wallet.proto:10-26).
``GetAccountRequest.identifier`` is a oneof of account_id / player_id; on the wire that is
two optional string fields, which is how it is declared here.
"""
from __future__ import annotations

from .builder import build_file, timestamp_class

FILE = "wallet/v1/wallet.proto"
PACKAGE = "wallet.v1"
SERVICE = "wallet.v1.WalletService"
TS = ".google.protobuf.Timestamp"
TX = ".wallet.v1.Transaction"

MESSAGES = {
    "CreateAccountRequest": [("player_id", 1, "string"), ("currency", 2, "string")],
    "CreateAccountResponse": [("account", 1, ".wallet.v1.Account")],
    "GetAccountRequest": [("account_id", 1, "string"), ("player_id", 2, "string")],
    "GetAccountResponse": [("account", 1, ".wallet.v1.Account")],
    "GetBalanceRequest": [("account_id", 1, "string")],
    "GetBalanceResponse": [("account_id", 1, "string"), ("balance", 2, "int64"), ("bonus", 3, "int64"),
                           ("total", 4, "int64"), ("withdrawable", 5, "int64"), ("currency", 6, "string")],
    "Account": [("id", 1, "string"), ("player_id", 2, "string"), ("currency", 3, "string"), ("balance", 4, "int64"),
                ("bonus", 5, "int64"), ("status", 6, "string"), ("created_at", 7, TS), ("updated_at", 8, TS)],
    "DepositRequest": [("account_id", 1, "string"), ("amount", 2, "int64"), ("idempotency_key", 3, "string"),
                       ("payment_method", 4, "string"), ("reference", 5, "string"), ("ip_address", 6, "string"),
                       ("device_id", 7, "string"), ("fingerprint", 8, "string")],
    "DepositResponse": [("transaction", 1, TX), ("new_balance", 2, "int64"), ("risk_score", 3, "int32")],
    "WithdrawRequest": [("account_id", 1, "string"), ("amount", 2, "int64"), ("idempotency_key", 3, "string"),
                        ("payout_method", 4, "string"), ("payout_details", 5, "string"), ("ip_address", 6, "string"),
                        ("device_id", 7, "string")],
    "WithdrawResponse": [("transaction", 1, TX), ("new_balance", 2, "int64"), ("risk_score", 3, "int32"),
                         ("payout_status", 4, "string")],
    "BetRequest": [("account_id", 1, "string"), ("amount", 2, "int64"), ("idempotency_key", 3, "string"),
                   ("game_id", 4, "string"), ("round_id", 5, "string"), ("game_category", 6, "string"),
                   ("ip_address", 7, "string"), ("device_id", 8, "string"), ("session_id", 9, "string")],
    "BetResponse": [("transaction", 1, TX), ("new_balance", 2, "int64"), ("risk_score", 3, "int32"),
                    ("real_deducted", 4, "int64"), ("bonus_deducted", 5, "int64")],
    "WinRequest": [("account_id", 1, "string"), ("amount", 2, "int64"), ("idempotency_key", 3, "string"),
                   ("game_id", 4, "string"), ("round_id", 5, "string"), ("bet_transaction_id", 6, "string"),
                   ("win_type", 7, "string"), ("metadata", 8, "string", "map:string:string")],
    "WinResponse": [("transaction", 1, TX), ("new_balance", 2, "int64")],
    "RefundRequest": [("account_id", 1, "string"), ("original_transaction_id", 2, "string"),
                      ("idempotency_key", 3, "string"), ("reason", 4, "string")],
    "RefundResponse": [("transaction", 1, TX), ("new_balance", 2, "int64")],
    "GetTransactionHistoryRequest": [("account_id", 1, "string"), ("limit", 2, "int32"), ("offset", 3, "int32"),
                                     ("types", 4, "string", "rep"), ("from", 5, TS), ("to", 6, TS),
                                     ("game_id", 7, "string")],
    "GetTransactionHistoryResponse": [("transactions", 1, TX, "rep"), ("total", 2, "int32"), ("has_more", 3, "bool")],
    "GetTransactionRequest": [("transaction_id", 1, "string")],
    "GetTransactionResponse": [("transaction", 1, TX)],
    "Transaction": [("id", 1, "string"), ("account_id", 2, "string"), ("idempotency_key", 3, "string"),
                    ("type", 4, "string"), ("amount", 5, "int64"), ("balance_before", 6, "int64"),
                    ("balance_after", 7, "int64"), ("status", 8, "string"), ("reference", 9, "string"),
                    ("game_id", 10, "string"), ("round_id", 11, "string"), ("risk_score", 12, "int32"),
                    ("created_at", 13, TS), ("completed_at", 14, TS)],
    "WalletError": [("code", 1, "string"), ("message", 2, "string"), ("details", 3, "string", "map:string:string")],
}

METHODS = [
    ("CreateAccount", "CreateAccountRequest", "CreateAccountResponse"),
    ("GetAccount", "GetAccountRequest", "GetAccountResponse"),
    ("GetBalance", "GetBalanceRequest", "GetBalanceResponse"),
    ("Deposit", "DepositRequest", "DepositResponse"),
    ("Withdraw", "WithdrawRequest", "WithdrawResponse"),
    ("Bet", "BetRequest", "BetResponse"),
    ("Win", "WinRequest", "WinResponse"),
    ("Refund", "RefundRequest", "RefundResponse"),
    ("GetTransactionHistory", "GetTransactionHistoryRequest", "GetTransactionHistoryResponse"),
    ("GetTransaction", "GetTransactionRequest", "GetTransactionResponse"),
]

# error codes (wallet.proto:233-241)
ERROR_CODES = ["INSUFFICIENT_BALANCE", "ACCOUNT_NOT_FOUND", "ACCOUNT_SUSPENDED", "DUPLICATE_TRANSACTION",
               "RISK_BLOCKED", "RISK_REVIEW", "INVALID_AMOUNT", "BONUS_RESTRICTION"]

M = build_file(FILE, PACKAGE, MESSAGES, services={"WalletService": METHODS},
               deps=["google/protobuf/timestamp.proto"])
Timestamp = timestamp_class()


def method_path(rpc: str) -> str:
    return f"/{SERVICE}/{rpc}"


def __getattr__(name):
    if name in M:
        return M[name]
    raise AttributeError(name)
