"""bench.py's film merge over RCCL, executed on the one-GPU box (VERDICT r05
item 5).  `bench.py --gpus 1 --rccl` starts torch.distributed.run with one rank
(as a child, before any GPU call), creates the `nccl` process group -- RCCL on
ROCm -- and reduces every frame's film with dist.reduce(SUM) onto rank 0: the
reference's Film::put merge (renderproc.cpp:142-149) as the 8-GPU run does it,
at world size 1.  The reduced film must equal the one-process film bit for bit,
and RCCL's own init log must show a one-rank communicator."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, name, rccl):
    out = str(tmp_path / name)
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    env['NCCL_DEBUG'] = 'INFO'
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '1', '--config', 'C1', '--steps', '2',
           '--warmup', '1', '--save-film', out, '--no-cpu-baseline', '--secondary', 'none']
    if rccl:
        cmd.append('--rccl')
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    log = p.stdout + p.stderr
    logdir = os.environ.get('MTSGPU_TEST_LOGDIR')
    if logdir:
        with open(os.path.join(logdir, 'rccl_world1_%s.log' % ('rccl' if rccl else 'plain')), 'w') as f:
            f.write(log)
    assert p.returncode == 0, log[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), np.load(out), log


def test_rccl_reduce_world1_equals_plain_film(tmp_path):
    r0, f0, _ = _bench(tmp_path, 'plain.npy', False)
    assert 'none' in r0['config']['parallelism']
    r1, f1, log = _bench(tmp_path, 'rccl.npy', True)
    assert r1['config']['world_size_reported'] == 1
    assert 'RCCL' in r1['config']['parallelism']
    assert r1['config']['samples_per_frame'] == 512 * 512 * 64
    # RCCL's communicator init line (NCCL_DEBUG=INFO): "... rank 0 nranks 1 ..."
    assert re.search(r'nranks 1\b', log), log[-3000:]
    assert f0.shape == f1.shape and f0.any()
    assert np.array_equal(f0.view(np.uint32), f1.view(np.uint32))
