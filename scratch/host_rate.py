"""Host-buffer entry points at batch scale: GiB/s of covered bytes for
ricrc_compute_batch / ricrc_compute_strided on pageable numpy buffers
(copy in, kernel, copy out), next to bench.py's pinned-tensor rate."""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "roce-sim_amd"))
from roce_icrc import IcrcEngine, synth  # noqa: E402

eng = IcrcEngine(0)
for n in (1 << 14, 1 << 17, 1 << 18):
    buf, stride, flen = synth.uniform_frames(n, 4096, seed=synth.SEED_CFG2)
    offs = (np.arange(n, dtype=np.uint64) * stride)
    lens = np.full(n, flen, np.uint32)
    cov = (flen - 4) * n
    for name, fn in (("strided", lambda: eng.compute_strided(buf, stride, flen, n)),
                     ("batch", lambda: eng.compute_batch(buf, offs, lens))):
        fn()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"n": n, "api": name, "MB": round(buf.nbytes / 1e6, 1),
                          "GiBps": round(cov / min(ts) / 2**30, 2)}), flush=True)
