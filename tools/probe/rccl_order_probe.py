"""Does RCCL order collectives of two communicators on one device in host launch order?
Stream A: long sleep kernel -> all_to_all on comm 0.  Stream B (issued after A in host order,
no dependency on A): all_to_all on comm 1 -> event. If B's event completes long before A's
sleep ends, the two communicators progress independently."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from igaming_platform_amd.parallel.exchange import rccl_comms  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
c0, c1 = rccl_comms(0, 1)
a, b = torch.cuda.Stream(), torch.cuda.Stream()
x0, y0 = torch.zeros(1 << 16, dtype=torch.uint8, device=dev), torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
x1, y1 = torch.zeros(1 << 16, dtype=torch.uint8, device=dev), torch.zeros(1 << 16, dtype=torch.uint8, device=dev)
for trial in range(3):
    torch.cuda.synchronize()
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    t0 = time.perf_counter()
    with torch.cuda.stream(a):
        torch.cuda._sleep(200_000_000)  # ~ 0.1 s
        c0.all_to_all(x0.data_ptr(), y0.data_ptr(), 1 << 16, a.cuda_stream)
        ea.record(a)
    with torch.cuda.stream(b):
        c1.all_to_all(x1.data_ptr(), y1.data_ptr(), 1 << 16, b.cuda_stream)
        eb.record(b)
    eb.synchronize()
    tb = time.perf_counter() - t0
    ea.synchronize()
    ta = time.perf_counter() - t0
    print(f"trial {trial}: comm1 done after {tb * 1e3:.2f} ms, comm0 (behind sleep) after {ta * 1e3:.2f} ms "
          f"-> {'INDEPENDENT' if tb < 0.5 * ta else 'SERIALISED'}", flush=True)
