#!/bin/bash
# Round 3 workload lines (through gpurun): lanes sweep on the 4K workload, config 4
# (batch1080), config 5 (16k-striped, 1 GPU), 16384^2 through the 4-lane pipeline.
set -u
cd ${GRAFT_REPO_ROOT:-.}
o=gpurun_out/r03l; mkdir -p $o
for l in 4 6 8; do
  timeout -k 10 200 python3 bench.py --lanes $l --frames 1536 --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > $o/lanes$l.json 2> $o/lanes$l.err || { tail -3 $o/lanes$l.err; exit 1; }
  echo "lanes $l: $(python3 -c "import json;d=json.loads(open('$o/lanes$l.json').read().strip().splitlines()[-1]);print(d['value'], d['host_cpu'])")"
done
timeout -k 10 300 python3 bench.py --workload batch1080 > $o/batch1080.json 2> $o/batch1080.err || { tail -3 $o/batch1080.err; exit 1; }
tail -c 700 $o/batch1080.json; echo
timeout -k 10 300 python3 bench.py --workload 16k-striped --steps 10 > $o/16k.json 2> $o/16k.err || { tail -3 $o/16k.err; exit 1; }
tail -c 500 $o/16k.json; echo
timeout -k 10 300 python3 bench.py --width 16384 --height 16384 --frames 16 --distinct 4 --steps 10 --no-cpu-baseline --d2h-steps 0 > $o/16k_pipe.json 2> $o/16k_pipe.err || { tail -3 $o/16k_pipe.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/16k_pipe.json').read().strip().splitlines()[-1])
print('16k pipeline', d['value'], {k:(round(v['avg_kernel_ms']*1e3,1), v['frac']) for k,v in d['stages_solo'].items()})"
true
