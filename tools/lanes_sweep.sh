cd $GRAFT_REPO_ROOT
for l in ${LANES:-2 3 4 6 8}; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --lanes $l > gpurun_out/lanes_$l.json 2>gpurun_out/lanes_$l.err || exit 1
  echo "lanes $l: $(python3 -c "import json;d=json.loads(open('gpurun_out/lanes_$l.json').read().strip().splitlines()[-1]);s=d['stages'];print(d['value'],[round(s[k]['avg_kernel_ms']*1000,1) for k in s])")"
done
