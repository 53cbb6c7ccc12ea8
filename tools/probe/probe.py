import os, sys, time, subprocess, sysconfig
here = os.path.dirname(os.path.abspath(__file__)); sys.path.insert(0, here)
import torch, pybind11
tl = os.path.join(os.path.dirname(torch.__file__), "lib")
so = os.path.join(here, "_probe" + sysconfig.get_config_var("EXT_SUFFIX"))
if not os.path.exists(so):
    subprocess.check_call(["hipcc","--offload-arch=gfx950","-O3","-fPIC","-shared","-std=c++17",
        "-I"+sysconfig.get_paths()["include"],"-I"+pybind11.get_include(),os.path.join(here,"probe.hip"),
        "-o",so,"-L"+tl,"-Wl,-rpath,"+tl])
import _probe
print("cuda avail", torch.cuda.is_available(), torch.cuda.get_device_name(0))
p = torch.cuda.get_device_properties(0); print(p)
x = torch.zeros(1000, device="cuda"); s = torch.cuda.current_stream().cuda_stream
_probe.launch(x.data_ptr(), x.numel(), s); torch.cuda.synchronize(); print("add ok", float(x.sum()))
o = torch.zeros(256, device="cuda"); _probe.mfma(o.data_ptr(), s); torch.cuda.synchronize(); print("mfma", o[:8].tolist(), bool((o==32).all()))
g = torch.cuda.CUDAGraph(); y = torch.zeros(1<<20, device="cuda")
with torch.cuda.graph(g):
    _probe.launch(y.data_ptr(), y.numel(), torch.cuda.current_stream().cuda_stream)
for _ in range(3): g.replay()
torch.cuda.synchronize(); print("graph ok", float(y[0]))
xc = torch.zeros(64, dtype=torch.int32, device="cuda"); _probe.xcc(xc.data_ptr(), 64, s); torch.cuda.synchronize(); print("xcc ids", xc.tolist()[:16])
torch.cuda.synchronize(); t=time.perf_counter()
for _ in range(1000): g.replay()
torch.cuda.synchronize(); print("graph replay us", (time.perf_counter()-t)*1e3)
t=time.perf_counter()
for _ in range(1000): _probe.launch(x.data_ptr(), x.numel(), s)
torch.cuda.synchronize(); print("eager launch us", (time.perf_counter()-t)*1e3)
print("mem", torch.cuda.mem_get_info())
