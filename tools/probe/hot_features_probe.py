#!/usr/bin/env python3
"""Diagnostic: the many-devices hot-account scenario of tests/test_engine_gpu.py repeated with
fresh engines; on a GetFeatures mismatch prints the whole GPU / CPU feature rows and the
registry's answer for the account."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))


def main() -> int:
    import test_engine_gpu as T
    from igaming_platform_amd.onnx import builders
    am = builders.build("gru", seq=100, hidden=64, layers=2).SerializeToString()
    bad = 0
    for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        g, c = T._engines(abuse_model=am)
        rng = np.random.default_rng(11 + rep)
        types = ["deposit", "withdraw", "bet", "win"]
        for step in range(3):
            acc = np.where(rng.random(1024) < 0.7, rng.integers(0, 2, 1024), rng.integers(2, 30, 1024))
            txs = [dict(account_id=f"acc-{int(a)}", amount=int(rng.integers(1, 300000)),
                        transaction_type=types[int(rng.integers(0, 4))], device_id=f"dev-{int(rng.integers(0, 400))}",
                        ip_address=f"10.3.{int(rng.integers(0, 20))}.{int(rng.integers(0, 20))}") for a in acc]
            g.score(txs, now=T.NOW + step * 20)
            c.score(txs, now=T.NOW + step * 20)
        for i in range(30):
            fg, fc = g.get_features(f"acc-{i}", now=T.NOW + 100), c.get_features(f"acc-{i}", now=T.NOW + 100)
            if fg["tx_count_1h"] != fc["tx_count_1h"]:
                bad += 1
                print("rep", rep, "acc", i, "registry", g.registry.resolve(f"acc-{i}", insert=False), flush=True)
                print(" gpu", fg, flush=True)
                print(" cpu", fc, flush=True)
                print(" again", g.get_features(f"acc-{i}", now=T.NOW + 100), flush=True)
        for e in (g, c):
            try:
                e.close()
            except Exception:
                pass
        print("rep", rep, "done", flush=True)
    print("mismatches", bad)
    return 0


if __name__ == "__main__":
    sys.exit(main())
