"""A/B of ragged-kernel builds (ROCE_ICRC_LIB) on cfg3 and homogeneous ragged
batches: kernel GiB/s (median of reps, HIP events) and parity vs the C oracle.
usage: python scratch/ulp_ab.py lib1.so lib2.so ...   (each run in a child process)"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def child(reps=30):
    sys.path.insert(0, str(ROOT / "roce-sim_amd"))
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np
    import torch
    from roce_icrc import IcrcEngine, synth
    from conftest import oracle_batch
    eng = IcrcEngine(0)
    s = torch.cuda.current_stream()
    cases = [("cfg3", synth.mixed_mtu_frames(1 << 20))]
    for mtu in (256, 512, 1024, 2048):
        n = (1 << 30) // (mtu + 44)
        buf, stride, flen = synth.uniform_frames(n, mtu, seed=5)
        offs = (np.arange(n, dtype=np.uint64) * np.uint64(stride))
        cases.append((f"u{mtu}", (buf, offs, np.full(n, flen, np.uint32))))
    res = []
    for name, (buf, offs, lens) in cases:
        n = offs.size
        want, _ = oracle_batch(buf, offsets=offs, lens=lens)
        trail = offs.astype(np.int64) + lens.astype(np.int64) - 4
        buf[(trail[:, None] + np.arange(4)[None, :]).reshape(-1)] = want.view(np.uint8)
        d = torch.from_numpy(buf).cuda()
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        out = torch.zeros(n, dtype=torch.int32, device="cuda")
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        cov = float((lens.astype(np.int64) - 4).sum())
        for mode in ("compute", "verify"):
            fn = (lambda: eng.compute_batch_dev(d, do, dl, n, out, stream=s.cuda_stream)) \
                if mode == "compute" else \
                (lambda: eng.verify_batch_dev(d, do, dl, n, ok, stream=s.cuda_stream))
            fn(); s.synchronize()
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s); fn(); e1.record(s); e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e-3)
            t = float(np.median(ts))
            if mode == "compute":
                bad = int((out.cpu().numpy().view(np.uint32) != want).sum())
            else:
                bad = int((ok.cpu().numpy() != 1).sum())
            res.append(f"{name:5s} {mode:7s} {cov / t / 2**30:8.1f} GiB/s  mismatches {bad}")
        del d
    print("\n".join(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        sys.exit(0)
    rc = 0
    for rnd in range(2):
        for lib in sys.argv[1:]:
            print(f"== {lib} (round {rnd})", flush=True)
            env = dict(os.environ, ROCE_ICRC_LIB=str(Path(lib).resolve()))
            r = subprocess.run([sys.executable, __file__, "--child"], env=env, timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)
