import os, sys, time
import numpy as np
order = sys.argv[1]
ROOT = "/root/repo"
sys.path.insert(0, ROOT + "/roce-sim_amd"); sys.path.insert(0, ROOT + "/tests"); sys.path.insert(0, ROOT + "/oracle")
def maps():
    return sorted({l.split()[-1].split('/')[-1] for l in open('/proc/self/maps') if 'amdhip' in l})
if order == "torch_first":
    import torch
from roce_icrc import IcrcEngine, synth
from roce_icrc.engine import load_library
load_library()
import torch
print(order, os.environ.get("ROCE_ICRC_LIB"), maps(), flush=True)
from conftest import oracle_batch
e = IcrcEngine(0)
n = 4096
buf, stride, flen = synth.uniform_frames(n, 4096)
want, _ = oracle_batch(buf, stride=stride, length=flen, n=n)
got, st = e.compute_strided(buf, stride, flen, n)
print("host api match:", bool((got == want).all()), flush=True)
try:
    d = torch.from_numpy(buf).cuda()
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    e.compute_strided_dev(d, stride, flen, n, out, stream=s.cuda_stream)
    torch.cuda.synchronize()
    print("dev api match:", bool((out.cpu().numpy().view(np.uint32) == want).all()), flush=True)
    n2 = 1 << 18
    buf2, stride, flen = synth.uniform_frames(n2, 4096)
    d2 = torch.from_numpy(buf2).cuda(); out2 = torch.zeros(n2, dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for r in range(3):
        ev[0].record(s); e.compute_strided_dev(d2, stride, flen, n2, out2, stream=s.cuda_stream); ev[1].record(s); ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1]); print("ms", ms, "GiB/s", (flen-4)*n2/ms/1e-3/2**30, flush=True)
except Exception as ex:
    print("torch path failed:", repr(ex)[:300], flush=True)
