# ad-hoc GPU sweep (used through gpurun): the bench under a few settings
mkdir -p gpurun_out
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
for cfg in "2 0" "2 1" "3 0" "3 1" "4 1" "2 0" "2 1" "3 0" "3 1" "4 1"; do set -- $cfg
  r=$(JPGE_LANES=$1 JPGE_NAP=$2 timeout -k 10 200 python bench.py --no-cpu-baseline 2>>gpurun_out/sweep_err.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
  echo "lanes=$1 nap=$2 $r"
done
