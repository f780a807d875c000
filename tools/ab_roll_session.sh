# A/B of rollout builds (tools/ab_build.py): 3 interleaved reps each, both the
# overlapped-streams value and the one-batch value of bench.py config 2.
O=gpurun_out/${AB_TAG:-abroll}; mkdir -p $O
for rep in 1 2 3; do
  for v in "$@"; do
    timeout -k 10 150 python tools/_ablib.py $v 4096 > $O/$(basename $v .so)_$rep.json 2> $O/$(basename $v .so)_$rep.err || exit 1
  done
done
for v in "$@"; do
  echo "$(basename $v .so) $(for rep in 1 2 3; do tail -1 $O/$(basename $v .so)_$rep.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.0f/%.0f" % (d["value"]/1e6, d["value_one_batch"]/1e6))'; done | tr '\n' ' ')"
done > $O/summary.txt
