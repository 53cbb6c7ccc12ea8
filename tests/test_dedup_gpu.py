"""Scorer-path dedup region (csrc/kernels/features.hip dedup_build_kernel): after one batch's
insert, every account of the batch is reachable from its hash slot by linear probing with its
first row and event count, fill / done are zero, unused slots are empty, and the batch's
hour word is set; each account's rows are in its list and the multi-event accounts in the
region's mlist. Compared with a plain numpy model of the same table."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M32 = 0xFFFFFFFF


def _mix32(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


@pytest.mark.parametrize("hot", [0.0, 0.5])
def test_dedup_region_after_insert(hot):
    import torch
    from igaming_platform_amd.features.device_store import DEDUP_LIST
    from igaming_platform_amd.ops import kernels as K
    from igaming_platform_amd.utils import benchkit
    from igaming_platform_amd.utils.synth import NOW0, make_requests
    dev = torch.device("cuda", 0)
    S = benchkit.build("cfg3", 1024, 4096, dev, hot_frac=hot)
    sc, store = S.scorer, S.store
    rng = np.random.default_rng(7)
    for n in (1024, 333):
        rows = make_requests(S.pop, n, rng, NOW0, hot_frac=hot)
        v = sc.slab_view(0, n)
        v[:] = rows
        sc._seq += 1
        sc._write_hdr(0, n, NOW0)
        nb = 16 + 48 * n
        sc.dev_slab[:nb].copy_(sc.host_slab[0][:nb])
        K.dedup_insert(store, sc.cfg_dev, sc.req, 1024, sc.hdr)
        torch.cuda.synchronize()
        cap, dmax = store.dcap, store.dmax
        reg = store.dbuf.view(-1, store.dregion)[sc._seq % 3].cpu().numpy()
        keys, first, count = reg[:cap], reg[cap:2 * cap], reg[2 * cap:3 * cap]
        fill, done = reg[3 * cap:4 * cap], reg[4 * cap:5 * cap]
        ctr = reg[5 * cap + cap * DEDUP_LIST + dmax:][:2]
        lists = reg[5 * cap:5 * cap + cap * DEDUP_LIST].reshape(cap, DEDUP_LIST)
        mlist = reg[5 * cap + cap * DEDUP_LIST:5 * cap + cap * DEDUP_LIST + dmax]
        slots = rows["slot"].astype(np.int64)
        want, rows_of = {}, {}
        for i, s in enumerate(slots):
            if s >= 0:
                f, c = want.get(int(s), (i, 0))
                want[int(s)] = (min(f, i), c + 1)
                rows_of.setdefault(int(s), []).append(i)
        assert (fill == 0).all() and (done == 0).all()
        assert int((keys >= 0).sum()) == len(want)
        assert (first[keys < 0] == 0x7FFFFFFF).all() and (count[keys < 0] == 0).all()
        for s, (f, c) in want.items():
            h = _mix32(s) & (cap - 1)
            while keys[h] != s:
                assert keys[h] != -1, f"account {s} not reachable from its hash slot"
                h = (h + 1) & (cap - 1)
            assert (first[h], count[h]) == (f, c), s
            if c <= DEDUP_LIST:  # the account's rows, in any order
                assert sorted(lists[h, :c].tolist()) == rows_of[s], s
        multi = {int(h) for h in np.nonzero(count >= 2)[0]}
        pairs = mlist[:2 * ctr[0]].reshape(-1, 2)  # {hash slot, account slot}
        assert ctr[0] == len(multi) and set(pairs[:, 0].tolist()) == multi
        assert (keys[pairs[:, 0]] == pairs[:, 1]).all()
        assert ctr[1] != 0
