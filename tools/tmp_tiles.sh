cd $GRAFT_REPO_ROOT
for v in 1; do
  echo "== SPK_NO_HALO=$v"
  SPK_NO_HALO=$v timeout -k 10 300 python tools/profile_steps.py --arch eres2netv2 --json gpurun_out/steps_nohalo.json > gpurun_out/steps_nohalo.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/steps_nohalo.txt | head -1
  grep -E "convs\.[01] " gpurun_out/steps_nohalo.txt | grep -E "layer[12]\.1\." 
done
