"""bench.py's N-rank launcher (the driver's `python bench.py --gpus N`), rehearsed
on CPU: the parent starts torch.distributed.run with N ranks before touching a
GPU, each rank renders its 8x8 tiles (here with the CPU oracle,
`--device cpu-oracle`; on the GPUs the HIP path with the same tile parameters)
and the films are reduced onto rank 0 (gloo here, RCCL on the GPUs).  The
reduced film must equal the single-process frame bit for bit, at 2, 4 and 8
ranks."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, gpus, name):
    out = str(tmp_path / name)
    env = dict(os.environ, OMP_NUM_THREADS='2')
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', str(gpus), '--device', 'cpu-oracle',
                        '--config', 'C1', '--size', '40x36x4', '--steps', '2', '--warmup', '1', '--save-film', out],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0]), np.load(out)


def test_multi_rank_launch_equals_single_process(tmp_path):
    r1, f1 = _bench(tmp_path, 1, 'f1.npy')
    assert r1['n_gpus'] == 1
    for n in (2, 4, 8):
        rn, fn = _bench(tmp_path, n, 'f%d.npy' % n)
        assert rn['n_gpus'] == n and rn['config']['world_size_reported'] == n
        assert rn['config']['samples_per_frame'] == r1['config']['samples_per_frame'] == 40 * 36 * 4
        assert np.array_equal(f1.view(np.uint32), fn.view(np.uint32)), n


def test_world_size_mismatch_fails(tmp_path):
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '4', '--device', 'cpu-oracle'],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and 'WORLD_SIZE' in p.stderr
