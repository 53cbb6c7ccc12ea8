"""MI355X-native iGaming risk platform (fraud scoring, LTV, bonus abuse, wallet).

HIP runtime options read once when the runtime initialises (the first GPU call), so they are
set here, at package import, unless the caller exported its own:

* ``HIP_FORCE_DEV_KERNARG=1``: kernel arguments in device memory. By default the runtime hands
  kernels their argument block in host memory, and every scalar load of an argument then costs
  ~1,900-3,100 cycles; in device memory 200-800 (rocprofv3 SmemLatency per kernel,
  profiles/r5/k/smem_latency.txt). Every kernel here reads its arguments on its critical path.
"""
import os

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
