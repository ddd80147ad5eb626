# Round 6: the per-packet path on the final library (6f21f47a): C latency of
# ricrc_compute_one / ricrc_icrc / bursts.
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 300 ./scratch/latency_c > $O/latency_c_r06.jsonl 2> $O/latency_c_r06.err
rc=$?; cat $O/latency_c_r06.jsonl; [ $rc -eq 0 ] || { tail -5 $O/latency_c_r06.err; exit $rc; }
