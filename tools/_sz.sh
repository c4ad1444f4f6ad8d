cd /root/repo
for cfg in "1260 10000" "5040 2500" "630 20000"; do
  set -- $cfg
  bash tools/prof_kernels.sh sz_$1 python3 tools/xs_one.py 0 $1 $2 > /dev/null || exit 1
  echo "== D=$1 N=$2"; grep xs_ gpurun_out/sz_$1_stats.txt
done
