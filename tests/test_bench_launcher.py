"""bench.py's own launcher: a bare `bench.py --gpus N` must start N rank
processes itself and report the world size the process group saw.  On CPU the
--cpu-plumbing mode runs the launcher, the gloo process group and the C4 exchange
(all-gather of per-rank embedding blocks) without any GPU work."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), *args], cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize('n', [1, 2])
def test_bench_self_launch_reports_world(n):
    line = _run('--gpus', str(n), '--steps', '2', '--warmup', '1', '--cpu-plumbing')
    assert line['n_gpus'] == n and line['world_size'] == n
    assert line['exchange_ok'] is True
    if n > 1:
        assert line['backend'] == 'gloo'
