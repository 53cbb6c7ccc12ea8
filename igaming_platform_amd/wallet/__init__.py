"""Wallet service: accounts, money movements with risk checks, double-entry ledger
(thin client of risk.v1; the reference's Go wallet service re-built in-process)."""
