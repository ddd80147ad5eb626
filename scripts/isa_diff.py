"""Compare the gfx950 assembly of two builds kernel by kernel.

usage: python scripts/isa_diff.py OLD.s NEW.s [substring]
Prints, per function whose name contains `substring`: instruction counts in
both builds, whether the bodies are identical (labels, comments and
directives stripped), and the VGPR / SGPR / spill counts of the new build.
(`make -C roce-sim_amd isa` writes the current build's .s files.)
"""
import re
import sys


def functions(path):
    text = open(path).read()
    out = {}
    for m in re.finditer(r"^(\S+):\s*; @\1\n(.*?)^\.Lfunc_end", text, re.S | re.M):
        body = []
        for line in m.group(2).split("\n"):
            line = line.split(";")[0].strip()
            if not line or line.startswith(".") or line.endswith(":"):
                continue
            body.append(re.sub(r"\.LBB\d+_\d+", "L", line))
        out[m.group(1)] = body
    meta = {}
    for m in re.finditer(r"\.set (\S+)\.(num_vgpr|num_sgpr|private_seg_size), (\d+)", text):
        meta.setdefault(m.group(1), {})[m.group(2)] = int(m.group(3))
    return out, meta


def main():
    old, _ = functions(sys.argv[1])
    new, meta = functions(sys.argv[2])
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    for name in sorted(set(old) | set(new)):
        if sub not in name:
            continue
        a, b = old.get(name), new.get(name)
        m = meta.get(name, {})
        print(f"{name[:90]:90s} old {len(a) if a else '-':>6} new {len(b) if b else '-':>6} "
              f"{'same' if a == b else 'DIFF'}  vgpr {m.get('num_vgpr', '?')} "
              f"sgpr {m.get('num_sgpr', '?')} scratch {m.get('private_seg_size', '?')}")


if __name__ == "__main__":
    main()
