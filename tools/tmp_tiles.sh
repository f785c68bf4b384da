cd $GRAFT_REPO_ROOT
for t in 256x128 128x256; do
  echo "== tile $t"
  SPK_X3_TILE=$t timeout -k 10 300 python tools/profile_steps.py --arch eres2netv2 --json gpurun_out/steps_t$t.json > gpurun_out/steps_t$t.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/steps_t$t.txt | head -2
  python tools/agg_steps.py gpurun_out/steps_t$t.json | head -14
done
