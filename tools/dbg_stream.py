import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from igaming_platform_amd.utils import benchkit
from igaming_platform_amd.utils.synth import NOW0, make_requests


def run(sizes, hot):
    dev = torch.device("cuda", 0)
    A = benchkit.build("cfg3", 512, 4096, dev, depth=3, history_batches=4, hot_frac=hot)
    B = benchkit.build("cfg3", 512, 4096, dev, depth=3, history_batches=4, hot_frac=hot)
    rng = np.random.default_rng(3)
    batches = [make_requests(A.pop, n, rng, NOW0, hot_frac=hot) for n in sizes]
    ref = [A.scorer.wait(A.scorer.submit(r, now=NOW0 + i), unpack=False)[0] for i, r in enumerate(batches)]
    sc = B.scorer
    sc.capture_pipelined()
    out = []
    for i, r in enumerate(batches):
        slot, done = sc.pipe_reserve()
        sc.pack(slot, r)
        sc.pipe_launch(len(r), NOW0 + i)
        out += [rows.numpy().copy() for _, rows, _ in done]
    out += [rows.numpy().copy() for _, rows, _ in sc.pipe_drain()]
    bad = [i for i, (a, b) in enumerate(zip(ref, out)) if not np.array_equal(a, b)]
    same = {n: bool(torch.equal(getattr(A.store, n), getattr(B.store, n))) for n in ("rt", "ring_ts", "hll")}
    print(sizes, "hot", hot, "mismatched batches", bad, "store equal", same, flush=True)


run([512, 512, 512, 512, 512, 512], 0.2)
run([512, 300, 512, 17, 512, 512, 200], 0.0)
run([512, 300, 512, 17, 512, 512, 200], 0.2)
run([17, 512, 512], 0.2)
run([512, 512, 512, 17], 0.2)
