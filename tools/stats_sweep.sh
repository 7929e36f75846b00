cd $GRAFT_REPO_ROOT
for w in 256 384 512 768 1024 1519; do
  echo "== stats wgs $w: $(JPGE_STATS_WGS=$w timeout -k 10 120 python3 tools/prof_frame.py --frames 16 --iters 64 2>&1 | tail -1)"
done
