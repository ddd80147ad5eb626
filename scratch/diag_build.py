"""Diagnostic library build (never shipped): a copy of roce-sim_amd/ under
/tmp/ricrc_diag whose strided, sorted-ragged, compact and small-frame kernels
record each workgroup's start and end (s_memrealtime, 100 MHz) into the
status buffer after its n status bytes (rounded up to 16): u64 pairs, one per
workgroup.  Output: scratch/libs/diag.so.  Read by scratch/tail_times.py."""
import re
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
D = Path("/tmp/ricrc_diag")
shutil.rmtree(D, ignore_errors=True)
shutil.copytree(ROOT / "roce-sim_amd", D / "roce-sim_amd", ignore=shutil.ignore_patterns("build", "*.so"))
shutil.copytree(ROOT / "include", D / "include")
k = D / "roce-sim_amd/csrc/icrc_kernels.hip"
s = k.read_text()
timer = """
struct DiagTimer {
  const IcrcArgs& a;
  uint64_t t0;
  __device__ explicit DiagTimer(const IcrcArgs& a_) : a(a_), t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ ~DiagTimer() {
    __syncthreads();
    if (threadIdx.x == 0 && a.status_out) {
      uint64_t* p = (uint64_t*)(a.status_out + ((a.n + 15u) & ~15u));
      p[2 * blockIdx.x] = t0;
      p[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
};
"""
s = s.replace("constexpr int kIcrcThreads = 1024;", timer + "constexpr int kIcrcThreads = 1024;", 1)
n = 0
for kern in ("icrc_strided_kernel", "icrc_ragged_mixed_kernel", "icrc_compact_kernel", "icrc_small_kernel"):
    pat = re.compile(r"(" + kern + r"\(IcrcArgs a\) \{\n)")
    s, c = pat.subn(r"\1  DiagTimer diag_timer(a);\n", s)
    n += c
assert n == 4, n
k.write_text(s)
r = subprocess.run(["make", "-s", "-j8", "-C", str(D / "roce-sim_amd"),
                    f"OUT={ROOT}/scratch/libs/diag.so", "BUILD=/tmp/ricrc_diag/build"])
sys.exit(r.returncode)
