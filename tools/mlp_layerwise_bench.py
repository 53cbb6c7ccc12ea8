#!/usr/bin/env python3
"""cfg 4 design comparison: the fused LTV chain kernel (one launch, 64-row
tiles, weights streamed from L2 per tile) against a layer-wise plan (one large-tile MFMA GEMM per
layer, 8192 x 512 activations staying in L2 / MALL between launches, the N=1 head last), both
captured in a hipGraph and replayed on one stream, same weights, same inputs; and the dedicated
layer-wise kernels (mlp_layers.hip).

Prints one JSON line per (design, precision, batch): microseconds per forward, predictions/s,
TFLOP/s, max |diff| against the chain. Usage: python tools/mlp_layerwise_bench.py [8192,16384]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FLOP_ROW = 2 * (256 * 512 + 3 * 512 * 512 + 512)


def _steps(rng):
    from igaming_platform_amd.models.plan import DenseStep, HeadStep
    steps = [DenseStep(n=512, k=k, act="relu", w_np=rng.normal(0, 0.05, (512, k)).astype(np.float32),
                       b_np=rng.normal(0, 0.1, 512).astype(np.float32)) for k in (256, 512, 512)]
    steps.append(HeadStep(n1=512, k=512, act1="relu", act2="none",
                          w1_np=rng.normal(0, 0.05, (512, 512)).astype(np.float32),
                          b1_np=rng.normal(0, 0.1, 512).astype(np.float32),
                          w2_np=rng.normal(0, 0.1, 512).astype(np.float32), b2=0.1))
    return steps


def _time_graph(torch, fn, reps=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    with torch.cuda.stream(s):  # replay() launches on the current stream: time it there
        for _ in range(reps):
            e0.record(s)
            g.replay()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        # back to back (the throughput a stream of batches sees: launch gaps overlap)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
        e1.synchronize()
    return float(np.median(ts)), g, e0.elapsed_time(e1) * 1e3 / reps


def main() -> int:
    import copy

    import torch
    from igaming_platform_amd.engine.runner import DeviceModel
    from igaming_platform_amd.models.plan import Plan, to_device
    from igaming_platform_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    steps = _steps(rng)
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    batches = [int(b) for b in (args[0] if args else "8192,16384").split(",")]
    out = []
    if "--trace" in sys.argv:  # per-phase wall clock of the layer kernels (blocks 0..63, wave 0)
        for precision in ("bf16", "fp32"):
            B = batches[0]
            lp = K.MlpLayerPack(steps, dev, split=precision == "fp32")
            lp.reserve(B)
            X = torch.from_numpy(rng.normal(0, 1, (B, 256)).astype(np.float32)).to(dev)
            ml = torch.zeros(B, device=dev)
            tr = torch.zeros((len(lp.layers), 64, 8), dtype=torch.int64, device=dev)
            for _ in range(3):
                K.mlp_layers(lp, B, X=X, ml=ml, trace=tr)
            torch.cuda.synchronize()
            t = tr.cpu().numpy().astype(np.float64) / 100.0  # 100 MHz ticks -> us
            for li in range(t.shape[0]):
                m = t[li]
                ph = {f"p{k}{k + 1}": round(float(np.median(m[:, k + 1] - m[:, k])), 2) for k in range(5)}
                r = dict(trace=True, precision=precision, batch=B, layer=li, start_skew_us=round(float(np.ptp(m[:, 0])), 2),
                         span_us=round(float(m[:, 5].max() - m[:, 0].min()), 2), **ph)
                out.append(r)
                print(json.dumps(r), flush=True)
    for precision in ("bf16", "fp32"):
        pk = K.MlpChainPack(steps, dev, split=precision == "fp32")
        plan = to_device(Plan(family="mlp", in_width=256, steps=copy.deepcopy(steps), out_width=1, ml_col=0,
                              metadata={}, input_name="input", output_name="output"), dev, precision)
        for B in batches:
            X = torch.from_numpy(rng.normal(0, 1, (B, 256)).astype(np.float32)).to(dev)
            ml = torch.zeros(B, device=dev)
            us_c, _g1, bb_c = _time_graph(torch, lambda: K.mlp_chain(pk, B, X=X, ml=ml))
            ref = ml.clone()
            lp = K.MlpLayerPack(steps, dev, split=precision == "fp32")  # noqa: F841
            lp.reserve(B)
            ml2 = torch.zeros(B, device=dev)
            us_k, _g3, bb_k = _time_graph(torch, lambda: K.mlp_layers(lp, B, X=X, ml=ml2))
            diff_k = float((ml2 - ref).abs().max())
            dm = DeviceModel(plan, dev, [B])
            res = {}

            def layerwise():
                res["y"] = dm.run(X, B)
            us_l, _g2, bb_l = _time_graph(torch, layerwise)
            diff = float((res["y"][:B, 0].float() - ref).abs().max())
            for name, us, bb, dd in (("chain", us_c, bb_c, 0.0), ("layerwise_generic", us_l, bb_l, diff),
                                     ("mlp_layers", us_k, bb_k, diff_k)):
                r = dict(design=name, precision=precision, batch=B, us=round(us, 2), us_back_to_back=round(bb, 2),
                         predictions_per_s_back_to_back=round(B / bb * 1e6),
                         predictions_per_s=round(B / us * 1e6), tflops=round(FLOP_ROW * B / us / 1e6, 1),
                         layers={"chain": "fused chain (mlp_fused.hip)",
                                 "layerwise_generic": "runner plan: " + plan.describe(),
                                 "mlp_layers": "mlp_layers.hip: 4 tile GEMMs + finish"}[name],
                         max_diff_vs_chain=dd)
                out.append(r)
                print(json.dumps(r), flush=True)
    with open(os.environ.get("OUT", "gpurun_out/mlp_layerwise.json"), "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
