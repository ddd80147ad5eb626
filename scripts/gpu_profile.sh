# GPU session: parity tests, bench, rocprofv3 kernel-trace stats, PMC traffic passes.
# usage: bash scripts/gpu_profile.sh <round tag, e.g. r01> [workload]
set -u
TAG=${1:-r01}
WL=${2:-cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
make -C oracle -s || exit 1
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== pytest -m gpu"
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -5 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
echo "== bench"
timeout -k 10 600 python bench.py --workload $WL > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cat $OUT/bench_$TAG.json; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_$TAG.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
echo "== rocprofv3 kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --workload $WL --no-cpu-baseline --no-e2e > $OUT/prof_$TAG.log 2>&1
rc=$?; tail -3 $OUT/prof_$TAG.log; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== pmc FETCH_SIZE"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf_$TAG -o run -- python3 $R/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmcf_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pmcf_$TAG.log; echo "pmcf rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo "== pmc WRITE_SIZE"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw_$TAG -o run -- python3 $R/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmcw_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pmcw_$TAG.log; echo "pmcw rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
# algorithmic bytes and the ceiling kernel's byte count from the bench line itself
ALG=$(python3 -c "import json; d=json.load(open('$OUT/bench_$TAG.json')); print(d['roofline']['alg_bytes_per_launch'])")
NP=$(python3 -c "import json; d=json.load(open('$OUT/bench_$TAG.json')); print(d['config']['packets_per_gpu'])")
if [ "$WL" = seg ]; then
  MR=$((NP * 4096))
  python3 scripts/pmc_traffic.py --fetch $OUT/pmcf_$TAG --write $OUT/pmcw_$TAG --workload seg \
    --packets $NP --frame-bytes 4140 --kernel segment_kernel --ceiling stream_copy_kernel \
    --ceiling-read-bytes $MR --alg-bytes $ALG --out $OUT/pmc_traffic_${TAG}_seg.json || exit 1
  KN=segment_kernel
else
  # the STREAM-read kernel reads the whole frame buffer: covered bytes + 4 B per frame
  BUF=$(python3 -c "import json; d=json.load(open('$OUT/bench_$TAG.json')); c=d['config']; print((c['covered_bytes_per_gpu'] + 4 * c['packets_per_gpu']) // 16 * 16)")
  KN=::icrc_
  # the sorted ragged verify kernel (cfg3 has no tiny frame: AUTO picks SORTED)
  [ "$WL" = cfg3 ] && KN="icrc_ragged_mixed_kernel<true>"
  # the compact ragged compute kernel with the ICRC output only (bench sets
  # RICRC_RAGGED_COMPACT; its checks run the verify form)
  [ "$WL" = ack ] && KN="icrc_compact_kernel<false, 1>"
  # FETCH_SIZE factor measured on this workload's own access pattern (scripts/fetch_calib.py)
  CAL=""
  CF=$R/profiles/r03b_fetch_calibration/$WL.json
  # cfg4's shard runs cfg2's kernel on cfg2-shaped frames: the same pattern
  [ "$WL" = cfg4 ] && CF=$R/profiles/r03b_fetch_calibration/cfg2.json
  if [ -f $CF ]; then
    F=$(python3 -c "import json; print(json.load(open('$CF'))['factor'])")
    CAL="--calibration $F --calibration-source ${CF#$R/}"
  fi
  python3 scripts/pmc_traffic.py --fetch $OUT/pmcf_$TAG --write $OUT/pmcw_$TAG --workload $WL \
    --packets $NP --frame-bytes 0 --ceiling-read-bytes $BUF --alg-bytes $ALG --kernel "$KN" $CAL \
    --out $OUT/pmc_traffic_${TAG}_$WL.json || exit 1
fi
python3 scripts/prof_summary.py $OUT/prof_$TAG $OUT/bench_$TAG.json "$KN" > $OUT/prof_summary_$TAG.txt || exit 1
cat $OUT/prof_summary_$TAG.txt
exit 0
