set -u
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for v in "SPK_DIAG_NO_RERUN=1" "SPK_X=0"; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1
  rc=$?; echo "[$v] $(tail -1 gpurun_out/ab_bench.log | cut -c1-140)"
  [ $rc -ne 0 ] && exit $rc
done
done
