"""Summarise rocprofv3 SQ/GRBM counter passes: per kernel, the mean of every
counter over its dispatches, plus the derived ratios used in DESIGN.md
(instructions per wave, busy fractions).

usage: python scripts/pmc_sq.py DIR [DIR ...] [--kernel NEEDLE]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import read_counters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="icrc_")
    a = ap.parse_args()
    agg = {}
    for d in a.dirs:
        for k, cs in read_counters(Path(d)).items():
            if a.kernel not in k:
                continue
            for c, v in cs.items():
                agg.setdefault(k, {})[c] = sum(v) / len(v)
    for k, cs in agg.items():
        print(k[:110])
        for c in sorted(cs):
            print(f"  {c:28s} {cs[c]:16.1f}")
        w = cs.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU"):
                if c in cs:
                    print(f"  {c + '/wave':28s} {cs[c] / w:16.1f}")
        cyc = cs.get("SQ_WAVE_CYCLES")
        if cyc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in cs:
                    print(f"  {c + '/WAVE_CYCLES':28s} {cs[c] / cyc:16.3f}")
        if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_LDS_IDX_ACTIVE" in cs:
            print(f"  {'LDS conflict frac':28s} {cs['SQ_LDS_BANK_CONFLICT'] / cs['SQ_LDS_IDX_ACTIVE']:16.3f}")


if __name__ == "__main__":
    main()
