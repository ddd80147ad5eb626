"""Turn rocprofv3 PMC passes of `bench.py` into profiles/pmc_traffic.json.

HBM bytes per launch of the ICRC kernel, from two separate counter passes
(FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), corrected as
/opt/skills/guides/MI355X_MICROARCH.md section HBM prescribes: FETCH_SIZE is
in KiB and on gfx950 under-reports wide streaming reads (1/2 for 16-B/lane
loads), so the read side is calibrated on the STREAM-read kernel that
bench.py runs over the SAME frame buffer (known byte count per launch).

usage: python scripts/pmc_traffic.py --fetch DIR --write DIR --workload cfg2 \
          --packets 1048576 --frame-bytes 4140 [--out profiles/pmc_traffic_cfg2.json]
       segmentation (seg): --kernel segment_kernel --ceiling stream_copy_kernel \
          --ceiling-read-bytes <MR bytes> --alg-bytes <MR + frames + 8/packet>
"""
import argparse
import csv
import hashlib
import json
from collections import defaultdict
from pathlib import Path


def read_counters(d: Path):
    """{kernel_name: {counter: [value per dispatch]}} from *counter_collection.csv."""
    res = defaultdict(lambda: defaultdict(list))
    files = list(Path(d).rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                res[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return res


def pick(res, needle):
    names = [k for k in res if needle in k]
    if not names:
        raise SystemExit(f"kernel matching {needle!r} not found in {list(res)[:5]}")
    return names[0]


def mean(xs):
    return sum(xs) / len(xs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--packets", type=int, required=True)
    ap.add_argument("--frame-bytes", type=int, required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--kernel", default="::icrc_")
    ap.add_argument("--ceiling", default="stream_read_kernel")
    ap.add_argument("--ceiling-read-bytes", type=int, default=0)
    ap.add_argument("--alg-bytes", type=int, default=0)
    ap.add_argument("--lib", default=str(Path(__file__).resolve().parent.parent / "roce-sim_amd" /
                                         "roce_icrc" / "libroceicrc.so"),
                    help="the library the passes ran (its sha256 binds the figure to the build)")
    ap.add_argument("--calibration", type=float, default=0.0,
                    help="FETCH_SIZE factor measured on this workload's own access pattern "
                         "(scripts/fetch_calib.py); default: the STREAM kernel of the same run")
    ap.add_argument("--calibration-source", default="")
    a = ap.parse_args()
    fr = read_counters(a.fetch)
    wr = read_counters(a.write)
    k_icrc = pick(fr, a.kernel)
    k_sr = pick(fr, a.ceiling)
    n, flen = a.packets, a.frame_bytes
    # bench.py's ceiling kernel reads the whole frame buffer (ICRC) or the MR (seg)
    sr_bytes = a.ceiling_read_bytes or (n * flen) // 16 * 16
    fetch_sr = mean(fr[k_sr]["FETCH_SIZE"]) * 1024
    calib = a.calibration or sr_bytes / fetch_sr
    calib_src = (a.calibration_source or "given") if a.calibration else \
        f"{a.ceiling} in the same run: known bytes read / FETCH_SIZE"
    fetch_icrc_raw = mean(fr[k_icrc]["FETCH_SIZE"]) * 1024
    write_icrc = mean(wr[pick(wr, a.kernel)]["WRITE_SIZE"]) * 1024
    fetch_icrc = fetch_icrc_raw * calib
    alg = a.alg_bytes or n * flen  # ICRC: C_i read + 4-B ICRC written = frame bytes per packet
    out = {
        "workload": a.workload,
        "packets": n,
        "kernel": k_icrc,
        "fetch_size_raw_bytes": round(fetch_icrc_raw),
        "fetch_calibration": round(calib, 4),
        "fetch_calibration_source": calib_src,
        "stream_kernel_calibration": round(sr_bytes / fetch_sr, 4),
        "fetch_bytes": round(fetch_icrc),
        "write_bytes": round(write_icrc),
        "traffic_bytes_per_launch": round(fetch_icrc + write_icrc),
        "alg_bytes_per_launch": alg,
        "traffic_over_alg": round((fetch_icrc + write_icrc) / alg, 4),
        "lib_sha256": hashlib.sha256(Path(a.lib).read_bytes()).hexdigest(),
        "dispatches": {"fetch_pass": len(fr[k_icrc]["FETCH_SIZE"]),
                       "write_pass": len(wr[pick(wr, a.kernel)]["WRITE_SIZE"])},
    }
    Path(a.out or f"profiles/pmc_traffic_{a.workload}.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
