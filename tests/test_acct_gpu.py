"""Native account RPCs on the GPU devices (engine/acct.py LtvNativeDevice / AbuseNativeDevice,
csrc/kernels/model_driver.hip): the LTV chain launched from the core's threads (pinned slot
slab in, pinned K9 rows out) and the abuse step (K1 feature rows + the GRU over the HBM event
rings) must answer exactly as the engine's Python path on the same GPU, and within float
tolerance of the CPU executor engine."""
import time

import numpy as np
import pytest

from tests.test_acct import NOW, _ask, _normalise, _populate, _python_answer, _requests

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_gpu_native_account_rpcs_equal_python_path(precision):
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.acct import AbuseNativeDevice, LtvNativeDevice
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    cfg = Config()
    cfg.gpu.buckets = [64, 512]
    cfg.ltv_model.precision = precision
    cfg.abuse_model.precision = precision
    lm = builders.build("ltv_mlp", n_features=64, width=128, layers=2).SerializeToString()
    am = builders.build("gru", seq=100, hidden=64, layers=2).SerializeToString()
    eng = RiskEngine(cfg, backend="gpu", capacity=256, ltv_model=lm, abuse_model=am)
    assert eng.acct is not None
    kinds = {type(d) for d in eng.acct.devices}
    assert kinds == {LtvNativeDevice, AbuseNativeDevice}  # the native path runs on the HIP devices
    ltv_dev = next(d for d in eng.acct.devices if isinstance(d, LtvNativeDevice))
    assert ltv_dev.g.chain is not None  # the fused chain: one recorded kernel per micro-batch
    ids = _populate(eng)
    reqs = _requests(ids)
    got = _ask(eng.acct.router, reqs)
    from igaming_platform_amd.proto import risk_v1 as P
    for (rpc, m), (b, e) in zip(reqs, got):
        assert e is None, e
        want = _python_answer(eng, rpc, m)
        if rpc == 3 and precision == "bf16":
            # bf16: the Python path may run the weight-stationary cluster GRU, the native step always
            # runs the batch-parallel kernel (different accumulation order)
            x, y = P.CheckBonusAbuseResponse.FromString(b), P.CheckBonusAbuseResponse.FromString(want)
            assert abs(x.abuse_score - y.abuse_score) < 2e-3 and list(x.linked_accounts) == list(y.linked_accounts)
            continue
        assert _normalise(rpc, b) == want, (rpc, m)
    st = eng.acct.router.stats(1)
    assert st["items"] == 2 * len(ids) and st["wait_errors"] == 0
    assert all(d.driver.submits > 0 for d in eng.acct.devices)
    eng.close()


def test_gpu_native_abuse_matches_cpu_engine():
    """GPU (K1 + split-MFMA GRU) vs CPU (C++ K1 twin + fp32 executor): same signals and linked
    accounts, scores within 1e-4."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.proto import risk_v1 as P
    am = builders.build("gru", seq=100, hidden=64, layers=2).SerializeToString()
    cfg = Config()
    cfg.gpu.buckets = [64, 512]
    g = RiskEngine(cfg, backend="gpu", capacity=256, abuse_model=am)
    c = RiskEngine(cfg, backend="cpu", capacity=256, abuse_model=am)
    ids = _populate(g)
    _populate(c)
    reqs = [x for x in _requests(ids) if x[0] == 3]
    a = _ask(g.acct.router, reqs)
    b = _ask(c.acct.router, reqs)
    for (x, _), (y, _) in zip(a, b):
        rx, ry = P.CheckBonusAbuseResponse.FromString(x), P.CheckBonusAbuseResponse.FromString(y)
        assert list(rx.signals) == list(ry.signals) and list(rx.linked_accounts) == list(ry.linked_accounts)
        assert rx.abuse_score == pytest.approx(ry.abuse_score, abs=1e-4)
    g.close()
    c.close()


@pytest.mark.parametrize("cluster_kernel", [False, True])
def test_gpu_native_abuse_cluster_kernel_option(cluster_kernel):
    """AbuseConfig.cluster_kernel: the 2 x 256 GRU's small steps on the split clusters
    (gru_wsx.hip, with the batch-parallel fallback graphs) or, by default, always on the
    batch-parallel split kernel - the same scores either way (both f32-faithful), no fallback."""
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.acct import AbuseNativeDevice
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.proto import risk_v1 as P
    am = builders.build("gru", seq=100, in_dim=16, hidden=256).SerializeToString()
    cfg = Config()
    cfg.gpu.buckets = [64, 512]
    cfg.abuse.cluster_kernel = cluster_kernel
    g = RiskEngine(cfg, backend="gpu", capacity=256, abuse_model=am)
    c = RiskEngine(cfg, backend="cpu", capacity=256, abuse_model=am)
    dev = next(d for d in g.acct.devices if isinstance(d, AbuseNativeDevice))
    assert any(gp.wsx_ok for gp in dev.gm.packs) == cluster_kernel
    assert (128 in dev.buckets) == cluster_kernel  # the cluster kernel's 128 / 256-row buckets
    ids = _populate(g)
    _populate(c)
    reqs = [x for x in _requests(ids) if x[0] == 3]
    a = _ask(g.acct.router, reqs)
    b = _ask(c.acct.router, reqs)
    for (x, _), (y, _) in zip(a, b):
        rx, ry = P.CheckBonusAbuseResponse.FromString(x), P.CheckBonusAbuseResponse.FromString(y)
        assert list(rx.signals) == list(ry.signals)
        assert rx.abuse_score == pytest.approx(ry.abuse_score, abs=1e-4)
    assert dev.driver.fallbacks == 0
    g.close()
    c.close()


def test_gpu_native_ltv_through_grpc_under_load():
    """Many concurrent PredictLTV calls over the native HTTP/2 server (open loop, native load
    generator): every call answered, micro-batched (fewer device steps than calls)."""
    from igaming_platform_amd.api.native_grpc import NativeRiskServer
    from igaming_platform_amd.config import Config
    from igaming_platform_amd.engine.risk_engine import RiskEngine
    from igaming_platform_amd.native import native
    from igaming_platform_amd.onnx import builders
    from igaming_platform_amd.proto import risk_v1 as P
    cfg = Config()
    cfg.gpu.buckets = [64, 512, 4096]
    lm = builders.build("ltv_mlp", n_features=256, width=512, layers=4).SerializeToString()
    eng = RiskEngine(cfg, backend="gpu", capacity=1024, ltv_model=lm)
    ids = _populate(eng)
    srv = NativeRiskServer(eng, port=0).start()
    try:
        payloads = [P.PredictLTVRequest(account_id=a).SerializeToString() for a in ids]
        r = native().grpc_load("127.0.0.1", srv.port, "/risk.v1.RiskService/PredictLTV", payloads, 20000.0, 1.0, 4, 256)
        assert r["errors"] == 0 and len(r["latency_ms"]) == r["sent"] > 15000
        st = eng.acct.router.stats(1)
        assert 0 < st["steps"] < st["items"]
        assert float(np.percentile(r["latency_ms"], 99)) < 50.0
    finally:
        srv.stop()
        eng.close()
    assert time.time() > NOW
