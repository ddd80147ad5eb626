# Round 5 session w: the per-packet path and the service beside batches on
# the final library (4c5b4f77): C latency of ricrc_compute_one / ricrc_icrc /
# bursts, and a cfg2 batch beside 0 / 1 / 4 / 10 threads calling ricrc_icrc.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 300 ./scratch/latency_c > $O/latency_c_r05w.jsonl 2> $O/latency_c_r05w.err
rc=$?; cat $O/latency_c_r05w.jsonl; [ $rc -eq 0 ] || { tail -5 $O/latency_c_r05w.err; exit $rc; }
timeout -k 10 400 python scripts/svc_contention.py > $O/svc_r05w.log 2>&1
rc=$?; tail -3 $O/svc_r05w.log; exit $rc
