cd $GRAFT_REPO_ROOT
for e in 0 1 2 3; do
  if [ $e = 0 ]; then L=3d-speaker_amd/lib/libspk_hip.so; else L=exp_libs/libspk_exp$e.so; fi
  echo "== EXP $e"
  SPK_HIP_LIB=$PWD/$L timeout -k 10 300 python tools/profile_steps.py --arch eres2netv2 --json gpurun_out/steps_exp$e.json > gpurun_out/steps_exp$e.txt 2>&1 || exit $?
  grep -E "layer[12]\.1\.convs" gpurun_out/steps_exp$e.txt
done
