import ctypes, os, sys, time
t_start = time.perf_counter()
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "ray-tracing-gpu_amd"))
mode = sys.argv[1]
T = {}
def mark(k): T[k] = round((time.perf_counter() - t_start) * 1e3, 2)
if mode == "torch":
    import torch
    mark("import_torch")
    torch.cuda.init(); torch.zeros(1, device="cuda"); torch.cuda.synchronize()
    mark("torch_cuda_init")
import rt_amd
mark("import_rt_amd")
L = rt_amd.lib()
mark("dlopen")
s = rt_amd.Scene(os.path.join(os.path.dirname(rt_amd.__file__), "..", "..", "tests", "golden", "scenes", "scene2.dat"), 1920, 1080, 3)
mark("parse_prepare")
c = rt_amd.Context(0)
mark("rt_create")
c.upload(s)
mark("upload")
img = c.render(s.frame)
mark("first_render")
img = c.render(s.frame)
mark("second_render")
print(mode, T)
