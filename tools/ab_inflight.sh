#!/bin/bash
# Interleaved bench.py runs at 3, 4 and 5 frames in flight (GPU box; cfg3 default workload).
# Round-1 close: 3 in flight 0.980-0.988 ms/step, 4: 0.991-1.012, 5: 0.986-1.001.
for r in 1 2 3 4; do for n in 3 4 5; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --inflight $n > /tmp/i.json 2>/dev/null || exit 1
  python3 -c "import json,sys;d=json.load(open('/tmp/i.json'));print(sys.argv[1], d['ms_per_step'])" "$r $n"
done; done
