import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
import tests.test_engine_gpu as T
from igaming_platform_amd.onnx import builders
from igaming_platform_amd.ops import kernels as K
if len(sys.argv) > 1:
    for name in ["test_gpu_engine_matches_cpu_engine_heuristic", "test_gpu_engine_with_stacked_model_close_to_cpu",
                 "test_gpu_ltv_matches_cpu"]:
        f = getattr(T, name, None)
        print("run", name, f is not None, flush=True)
        if f: f()
m = builders.build("gru", seq=100, hidden=256, layers=2).SerializeToString()
g, c = T._engines(abuse_model=m)
ev = [dict(account_id=f"acc-{i % 10}", amount=100 * (i % 13) + 1, transaction_type=["deposit", "bet"][i % 2], device_id=f"d{i % 3}", ts=T.NOW - 500 + i) for i in range(150)]
g.ingest_events(ev); c.ingest_events(ev)
ag = g.abuse.gpu[0] if hasattr(g.abuse, "gpu") and g.abuse.gpu else None
print("ag", type(ag), flush=True)
for i in range(3):
    a = g.check_bonus_abuse(f"acc-{i}", now=T.NOW); b = c.check_bonus_abuse(f"acc-{i}", now=T.NOW)
    print(i, a.model_score, b.model_score, "ws_failed", ag.gp.ws_failed() if ag else None, flush=True)
if ag:
    gp = ag.gp
    print("ws", gp._ws["clusters"] if gp._ws else None, len(gp._ws_old), flush=True)
    slots = torch.tensor([0, 1, 2, -1], dtype=torch.int32, device=ag.device)
    for ws in (1, 0):
        out = torch.zeros(4, device=ag.device)
        tr = torch.zeros(64 * 8 + 4, dtype=torch.int64, device=ag.device)
        K.gru(gp, 4, ag.T, out=out, store=ag.store, slots=slots, ws=ws, ws_trace=tr)
        torch.cuda.synchronize()
        print("eager ws", ws, out.tolist(), "failed", gp.ws_failed(), "trace0", tr[:6].tolist(), flush=True)
