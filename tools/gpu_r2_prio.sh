set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 | cut -c1-260 | sed "s/^/base $i /" >> gpurun_out/prio_ab.log || exit 1
  FM_FRONT_PRIO=1 timeout -k 10 120 python bench.py --steps 300 --warmup 30 | cut -c1-260 | sed "s/^/prio $i /" >> gpurun_out/prio_ab.log || exit 1
done
echo done
