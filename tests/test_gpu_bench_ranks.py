"""bench.py's N-rank path on the GPU: the launcher starts torch.distributed.run,
each rank renders its 8x8 tiles through the HIP library and the films are
reduced onto rank 0.  The box has one GPU, so the ranks share it
(`--share-device`: every rank on GPU 0, the reduce over gloo through host
memory, since RCCL refuses two ranks on one device); the tile decomposition,
the per-rank HIP renders, the barriers and the merge are the ones an 8-GPU node
runs.  The reduced film must equal the one-process frame bit for bit (box
filter: ranks own disjoint pixels)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, gpus, name, cfg, size):
    out = str(tmp_path / name)
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', str(gpus), '--config', cfg, '--size', size,
           '--steps', '2', '--warmup', '1', '--save-film', out, '--no-cpu-baseline', '--secondary', 'none']
    if gpus > 1:
        cmd.append('--share-device')
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), np.load(out)


@pytest.mark.parametrize('cfg,size', [('C1', '96x72x16'), ('C3', '96x64x8')])
def test_ranks_on_gpu_equal_one_process(tmp_path, cfg, size):
    r1, f1 = _bench(tmp_path, 1, 'f1.npy', cfg, size)
    w, h, spp = (int(x) for x in size.split('x'))
    assert r1['config']['samples_per_frame'] == w * h * spp
    for n in (2, 4):
        rn, fn = _bench(tmp_path, n, 'f%d.npy' % n, cfg, size)
        assert rn['n_gpus'] == n and rn['config']['world_size_reported'] == n
        assert 'rehearsal' in rn['device']
        assert np.array_equal(f1.view(np.uint32), fn.view(np.uint32)), (cfg, n)
