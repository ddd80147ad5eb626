"""A/B variant library (never shipped): a copy of roce-sim_amd/ under
/tmp/ricrc_var_<name> with literal text substitutions applied to one source,
built to scratch/libs/<name>.so.

usage: python scratch/variant_build.py <name> <csrc file> '<old>' '<new>' ['<old>' '<new>' ...]"""
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
name, src = sys.argv[1], sys.argv[2]
pairs = sys.argv[3:]
assert len(pairs) % 2 == 0 and pairs, "old/new pairs"
D = Path(f"/tmp/ricrc_var_{name}")
shutil.rmtree(D, ignore_errors=True)
shutil.copytree(ROOT / "roce-sim_amd", D / "roce-sim_amd", ignore=shutil.ignore_patterns("build", "*.so"))
shutil.copytree(ROOT / "include", D / "include")
f = D / "roce-sim_amd/csrc" / src
s = f.read_text()
for old, new in zip(pairs[::2], pairs[1::2]):
    assert s.count(old) == 1, f"{old!r} occurs {s.count(old)} times"
    s = s.replace(old, new)
f.write_text(s)
r = subprocess.run(["make", "-s", "-j8", "-C", str(D / "roce-sim_amd"), f"OUT={ROOT}/scratch/libs/{name}.so",
                    f"BUILD={D}/build"], capture_output=True, text=True)
print(r.stdout[-2000:], r.stderr[-2000:] if r.returncode else "")
sys.exit(r.returncode)
