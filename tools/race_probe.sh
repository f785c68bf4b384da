set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/race_probe4.py eres2netv2 2>&1 | grep -v amdgpu.ids
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/race_probe3.py eres2netv2 2>&1 | grep -v amdgpu.ids
