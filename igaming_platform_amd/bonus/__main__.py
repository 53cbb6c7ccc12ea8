"""Bonus rules CLI: ``python -m igaming_platform_amd.bonus validate|list|eligible ...``."""
from __future__ import annotations

import argparse
import json
import os

from .engine import BonusEngine, PlayerInfo, load_rules_file

DEFAULT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs", "bonus_rules.yaml")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["validate", "list", "eligible"])
    ap.add_argument("--config", default=os.environ.get("CONFIG_PATH", DEFAULT))
    ap.add_argument("--age-days", type=int, default=0)
    ap.add_argument("--deposits", type=int, default=0)
    ap.add_argument("--segment", default="")
    ap.add_argument("--country", default="")
    ap.add_argument("--promo", default="")
    a = ap.parse_args(argv)
    rules = load_rules_file(a.config)
    if a.cmd == "validate":
        print(f"ok: {len(rules)} rules")
    elif a.cmd == "list":
        for r in rules:
            print(json.dumps(dict(id=r.id, type=r.type, active=r.active, name=r.name)))
    else:
        from ..wallet.repository import BonusRepository, Database
        be = BonusEngine(rules, BonusRepository(Database()),
                         players=lambda acc: PlayerInfo(acc, a.age_days, a.deposits, a.segment, a.country))
        for r in be.eligible("cli", promo_code=a.promo):
            print(r.id)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
