cd $GRAFT_REPO_ROOT
for f in 768 1536 384; do
  timeout -k 10 300 python3 bench.py --frames $f --steps 6 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/fr.json 2> gpurun_out/fr.err || exit 1
  echo "== frames $f: $(python3 -c "import json;d=json.loads(open('gpurun_out/fr.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
