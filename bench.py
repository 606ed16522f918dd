#!/usr/bin/env python3
"""bench.py -- Msamples/s of the MI355X `path` integrator on BASELINE config C2.

Workload (BASELINE.json configs[1]): Cornell box, 1280x720, 512 spp, sobol,
path maxDepth=-1 rrDepth=5, box filter.  One step = one full frame
(471,859,200 samples = one pass of the hot path over the frame) rendered into
an HBM-resident film; with N GPUs the frame's rows are sharded (8-row blocks,
interleaved over ranks) and the films are reduced to rank 0 with one RCCL
reduce over xGMI (the reference's Film::put merge, renderproc.cpp:142-149).
Total work is fixed as N grows: scaling "strong".

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 through
torch.distributed.run (one process per GPU, RCCL backend).
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402  (loads the HIP runtime first; libmtsgpu shares it)
import torch.distributed as dist  # noqa: E402

from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import film_border, scenes  # noqa: E402
from mitsuba_amd.distributed import ROW_BLOCK, RowSharding  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
WORKLOADS = {
    'C1': 'C1: Cornell box 512x512 64 spp (plumbing config)',
    'C2': 'C2: Cornell box (32 tris, diffuse, area light), path maxDepth=-1 rrDepth=5, sobol, box filter',
    'C3': 'C3: matpreview (69k-tri object, roughconductor GGX a=0.1 Cu, diffuse checker ground, 1024x512 '
          'envmap only), path maxDepth=-1 rrDepth=5, sobol, box filter',
    'C4': 'C4: atrium (195k tris, 24 fluted columns, roughdielectric GGX a=0.2 eta=1.5 on ~30% of meshes, '
          'diffuse elsewhere, 4 area lights) 1280x720 256 spp, path maxDepth=-1 rrDepth=5, sobol, box filter',
    'C5': 'C5: matpreview with the object in roughplastic GGX, checkerboard-textured alpha (0.05/0.3) -> '
          '2D rough-transmittance slice (50 alpha x 100 theta) per shading point, 1024x512 envmap, 1024 spp, '
          'path maxDepth=-1 rrDepth=5, sobol, box filter',
}


def algorithmic_bytes_per_sample(st, scene_prims, num_emitters):
    """SURVEY.md 8(d) no-reuse model in this build's HBM layout:
    64 B per BVH2 node visit (both child boxes), 48 B per TriAccel test,
    per hit 116 B (prim record 16 + vertices 36 + normals 36 + UV tangent 12 +
    shape record 16) + 80 B BSDF record, per emitter sample the two CDF binary
    searches + emitter record 48 + light triangle 52, 4 B per Sobol
    direction-number word, 20 B film write per pixel (amortised over spp)."""
    n = max(1, st['samples'])
    log2 = lambda x: math.ceil(math.log2(max(2, x + 1)))
    nee_bytes = 4 * (log2(num_emitters) + 1) + 48 + 4 * (log2(64) + 2) + 16 + 36
    b = (64.0 * st['node_visits'] + 48.0 * st['tri_tests'] + (116.0 + 80.0) * st['hits'] +
         nee_bytes * st['nee_samples'] + 4.0 * st['sobol_reads'])
    return b / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='C2')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-threads', type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    scene, integ = scenes.build(args.config, rfilter='box')
    W, H, spp = scene.sensor.width, scene.sensor.height, integ.sampleCount
    ctx = Context(dev)
    t_up = time.time()
    ctx.upload(scene)
    upload_s = time.time() - t_up
    b = film_border(integ.rfilter, integ.rfilterParam)
    film = torch.zeros(((H + 2 * b) * (W + 2 * b) * 5,), dtype=torch.float32, device='cuda')
    stream = torch.cuda.current_stream().cuda_stream
    shard = RowSharding(rank, world, ROW_BLOCK)
    row = shard.row_params()

    def step():
        st = ctx.render_device(integ, film.data_ptr(), stream, row=row)
        shard.reduce(film, dist)
        return st

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    samples_rank = 0
    for _ in range(args.steps):
        st = step()
        kernel_ms.append(st['kernel_ms'])
        samples_rank += st['samples']
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
    s = torch.tensor([samples_rank], dtype=torch.float64, device='cuda')
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
    elapsed_max = float(t.item())
    total_samples = float(s.item())
    frame_samples = W * H * spp
    assert int(total_samples) == frame_samples * args.steps, (total_samples, frame_samples)

    if rank == 0:
        value = total_samples / elapsed_max / 1e6
        # roofline: traversal counters from a bounded stats pass (1/16 of the rows), always
        # through the BVH: tiny scenes' linear TriAccel scan (an implementation choice that
        # reads every record from the scalar cache) must not inflate the workload's bytes
        os.environ['MTSGPU_NO_SCAN'] = '1'
        try:
            _, _, sst = ctx.render(integ, row=(ROW_BLOCK, 16, 0), traversal_stats=True)
        finally:
            os.environ.pop('MTSGPU_NO_SCAN', None)
        bps = algorithmic_bytes_per_sample(sst, scene.num_triangles, len(scene.emitters))
        avg_kernel_s = (sum(kernel_ms) / len(kernel_ms)) / 1e3
        per_launch_samples = samples_rank / max(1, len(kernel_ms))
        achieved = bps * per_launch_samples / avg_kernel_s / 1e9
        roofline = {'bound': 'hbm', 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
                    'frac': round(achieved / HBM_PEAK_GBPS, 5), 'traffic': measured_traffic(args.config),
                    'algorithmic_bytes_per_sample': round(bps, 1),
                    'kernel_ms_avg': round(avg_kernel_s * 1e3, 3)}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(scene, integ, args.cpu_threads)
        out = {
            'metric': 'Msamples/s (and s/frame) at 512 spp, 1280x720', 'value': round(value, 2),
            'unit': 'Msamples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(elapsed_max / args.steps * 1e3, 2), 'higher_is_better': True,
            'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': {'workload': WORKLOADS.get(args.config, args.config), 'width': W, 'height': H, 'spp': spp,
                       'samples_per_frame': frame_samples, 'parallelism': 'rows sharded x%d + RCCL film reduce' % world,
                       's_per_frame': round(elapsed_max / args.steps, 4), 'scene_upload_s': round(upload_s, 3)},
            'roofline': roofline,
            'cpu_baseline': cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def measured_traffic(cfg):
    """HBM bytes per launch of the path kernel on this workload from the committed
    PMC passes (profiles/<round>_traffic_<cfg>.json, written by
    tools/traffic_summary.py from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md); None when no summary exists."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', '*_traffic_%s.json' % cfg)))
    if not files:
        return None
    t = json.load(open(files[-1]))
    return {'bytes_per_launch': t['hbm_bytes_per_launch'], 'unit': 'B', 'source': os.path.basename(files[-1])}


def cpu_baseline(scene, integ, threads):
    """The CPU restatement (oracle, OpenMP over host cores) on a bounded sample of
    the same workload: the full 1280x720 frame at 256 spp (first 256 Sobol samples
    of every pixel)."""
    import oracle.binding as ob
    import copy
    threads = threads or min(16, os.cpu_count() or 1)
    it = copy.copy(integ)
    it.sampleCount = 256
    t0 = time.perf_counter()
    _, _, st = ob.render(scene, it, libm_mode=0, threads=threads)
    dt = time.perf_counter() - t0
    return {'value': round(st['samples'] / dt / 1e6, 3), 'unit': 'Msamples/s', 'cores': threads, 'kind': 'port',
            'sample': '%dx%d at 256 spp (%d samples, %.1f s)' % (scene.sensor.width, scene.sensor.height,
                                                                 st['samples'], dt)}


if __name__ == '__main__':
    main()
