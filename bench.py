#!/usr/bin/env python3
"""bench.py -- Msamples/s of the MI355X `path` integrator on BASELINE config C2,
and on C3 (matpreview, BASELINE's second north-star scene), C4 (the 200k-triangle
atrium BASELINE names for tile sharding), C5 (roughplastic with the
rough-transmittance lookup) and C2g (C2 with the reference's default gaussian
reconstruction filter) in the same run, as the line's `secondary` blocks (one
per config, each with its own value, ms_per_step, roofline and CPU baseline).

Workload (BASELINE.json configs[1]): Cornell box, 1280x720, 512 spp, sobol,
path maxDepth=-1 rrDepth=5, box filter.  One step = one full frame
(471,859,200 samples = one pass of the hot path over the frame) rendered into
an HBM-resident film; with N GPUs the frame's 8x8 pixel tiles are dealt
round-robin over the ranks (tile t to rank t % N, MTSGPU_FLAG_TILE_SHARD: every
rank keeps whole tiles at any N, and the 14,400 tiles of a 1280x720 frame
split evenly over 1-8 ranks) and the films are summed onto rank 0 with one RCCL reduce over xGMI (the
reference's Film::put merge, renderproc.cpp:142-149).  Total work is fixed as
N grows: scaling "strong".

Launch: `python bench.py [--gpus N --steps K --warmup W]`.  With N > 1 and no
torch.distributed environment, this process starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child
(one process per GPU, RCCL backend) before touching the GPU, and exits with
its status; under torch.distributed.run WORLD_SIZE must equal N.

`--device cpu-oracle` is a launcher rehearsal for machines without a GPU (the
CPU test suite): each rank renders its tiles with the CPU oracle and the films
are reduced over gloo.  It is never selected implicitly; the GPU path fails
loudly when the HIP library or the GPU is missing.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BASELINE_METRIC = 'Msamples/s (and s/frame) at 512 spp, 1280×720; 1/2/4/8 MI355X + CPU ref'
WORKLOADS = {
    'C1': 'C1: Cornell box 512x512 64 spp (plumbing config)',
    'C2': 'C2: Cornell box (32 tris, diffuse, area light), path maxDepth=-1 rrDepth=5, sobol, box filter',
    'C3': 'C3: matpreview (69k-tri object, roughconductor GGX a=0.1 Cu, diffuse checker ground, 1024x512 '
          'envmap only), path maxDepth=-1 rrDepth=5, sobol, box filter',
    'C4': 'C4: atrium (195k tris, 24 fluted columns, roughdielectric GGX a=0.2 eta=1.5 on ~30% of meshes, '
          'diffuse elsewhere, 4 area lights) 1280x720 256 spp, path maxDepth=-1 rrDepth=5, sobol, box filter',
    'C2g': 'C2g: C2 with the reference\'s default reconstruction filter (gaussian stddev 0.5, 5x5 footprint), '
           'the film gathered per pixel in a fixed order (film_gather)',
    'C5': 'C5: matpreview with the object in roughplastic GGX, checkerboard-textured alpha (0.05/0.3) -> '
          '2D rough-transmittance slice (50 alpha x 100 theta) per shading point, 1024x512 envmap, 1024 spp, '
          'path maxDepth=-1 rrDepth=5, sobol, box filter',
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='C2')
    ap.add_argument('--size', default=None, help='WxHxSPP override (launcher rehearsals and tests only)')
    ap.add_argument('--device', default='gpu', choices=['gpu', 'cpu-oracle'])
    ap.add_argument('--save-film', default=None, help='rank 0 writes the reduced film (.npy) after the last step')
    ap.add_argument('--share-device', action='store_true',
                    help='every rank on GPU 0, films reduced over gloo through host memory: a one-GPU rehearsal '
                         'of the N-rank path (tests only; never a measurement)')
    ap.add_argument('--rccl', action='store_true',
                    help='create the nccl (RCCL) process group and reduce the film over it even at --gpus 1 '
                         '(launched through torch.distributed.run --nproc-per-node 1): executes the RCCL merge '
                         'path on a one-GPU box')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-threads', type=int, default=0)
    ap.add_argument('--secondary', default='C3,C4,C5,C2g',
                    help="further workloads timed in the same run (comma-separated), each emitted as a block of "
                         "the line's `secondary` object; 'none' to skip")
    return ap.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """Start one process per GPU through torch.distributed.run (as a child: this
    process has not touched the GPU and never execs) and return its exit code;
    None when this process is already a rank or N == 1."""
    world_env = os.environ.get('WORLD_SIZE')
    if world_env is not None:
        if int(world_env) != args.gpus:
            sys.exit('bench.py: --gpus %d but WORLD_SIZE=%s; launch with --nproc-per-node %d' %
                     (args.gpus, world_env, args.gpus))
        return None
    if args.gpus == 1 and not args.rccl:
        return None
    if args.gpus < 1:
        sys.exit('bench.py: --gpus must be >= 1')
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env.setdefault('OMP_NUM_THREADS', '1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args.gpus),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    return subprocess.call(cmd, env=env)


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


def lib_sha256(path=None):
    """sha256 of the libmtsgpu.so this run loads: the build a profile was taken on."""
    import hashlib
    if path is None:
        sys.path.insert(0, REPO)
        from pkgimport import mitsuba_amd
        mitsuba_amd()
        from mitsuba_amd.integrator import LIB_PATH
        path = LIB_PATH
    h = hashlib.sha256()
    with open(path, 'rb') as f:
        for chunk in iter(lambda: f.read(1 << 20), b''):
            h.update(chunk)
    return h.hexdigest()


def measured_profile(kind, cfg):
    """The newest committed summary profiles/<round>_<kind>_<cfg>.json, written
    by tools/traffic_summary.py (traffic: HBM bytes per launch and per sample from
    separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes; valu: VALU instructions per
    sample, shader clock, VALU-busy and wait fractions from one SQ pass); None
    when none exists."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_%s_%s.json' % (kind, cfg))))
    if not files:
        return None
    t = json.load(open(files[-1]))
    t['source'] = os.path.basename(files[-1])
    return t


def valu_calibration():
    """The newest committed VALU calibration (tools/valu_calib.hip -> tools/calib_summary.py
    -> profiles/<round>_valu_calib.json): the SIMD-cycles per wave64 VALU instruction a
    pure-VALU kernel sustains at saturation, measured with the same SQ counters as the
    path kernel's pass; None when none is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_valu_calib.json')))
    if not files:
        return None
    c = json.load(open(files[-1]))
    c['source'] = os.path.basename(files[-1])
    return c


def roofline_line(bps, launch_samples, kernel_s, cfg, lib_hash=None):
    """The dominant kernel's roofline, from the live kernel time of this run and
    per-sample work measured once per build by rocprofv3 (profiles/<round>_*):
      hbm   -- measured HBM bytes per sample (separate FETCH_SIZE / WRITE_SIZE
               passes, FETCH doubled per MI355X_MICROARCH.md) x samples / time,
               against the 8 TB/s HBM3E peak;
      valu  -- wave64 VALU instructions per sample (SQ_INSTS_VALU of the SQ pass)
               x samples / time, against the calibrated issue peak: 1024 SIMDs x
               the pass's shader clock / the SIMD-cycles per VALU instruction that
               a pure-VALU kernel sustains at saturation (profiles/r*_valu_calib
               .json: 4.19 at 8 waves/SIMD, for v_fma_f32 and for the packed v_pk_*
               alike).  Beside it: `busy` (4 x SQ_ACTIVE_INST_VALU quad-cycles per
               SIMD-cycle; the calibration kernel saturates at 0.955) and
               `spec_lane_issue` (f32 lane-ops against the 157 TF spec rate of 32
               lane-FMAs per SIMD-cycle, which only packed instructions reach: the
               calibration measures 15.3 unpacked vs 30.5 packed lane-ops per cycle).
    `bound` is the resource with the larger calibrated fraction; the other is kept,
    as is the SURVEY.md 8(d) no-reuse byte model (`hbm_model`), and, when committed,
    the stall attribution (profiles/r*_stalls_<cfg>.json: per-kind instruction
    counts and latencies)."""
    traffic = measured_profile('traffic', cfg)
    valu = measured_profile('valu', cfg)
    stalls = measured_profile('stalls', cfg)
    calib = valu_calibration()
    # a per-sample profile only describes the build it was taken on (tools/prof_round.sh
    # stamps each with the library's sha256): another build's profile gives no `frac`
    stale = []
    for name, prof in (('traffic', traffic), ('valu', valu)):
        if prof is not None and prof.get('lib_sha256') != lib_hash:
            stale.append('%s (%s, built from %s)' % (prof['source'], name, (prof.get('lib_sha256') or 'no stamp')[:12]))
    if stale:
        traffic = traffic if traffic and traffic.get('lib_sha256') == lib_hash else None
        valu = valu if valu and valu.get('lib_sha256') == lib_hash else None
    model = {'achieved': round(bps * launch_samples / kernel_s / 1e9, 2), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
             'frac': round(bps * launch_samples / kernel_s / 1e9 / HBM_PEAK_GBPS, 5),
             'algorithmic_bytes_per_sample': round(bps, 1),
             'note': 'no-reuse model: BVH nodes 64 B, TriAccel 48 B, hit/NEE/Sobol/film bytes (bench.py)'}
    hbm = None
    if traffic and traffic.get('hbm_bytes_per_sample'):
        a = traffic['hbm_bytes_per_sample'] * launch_samples / kernel_s / 1e9
        hbm = {'achieved': round(a, 2), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s', 'frac': round(a / HBM_PEAK_GBPS, 5),
               'bytes_per_sample': round(traffic['hbm_bytes_per_sample'], 1),
               'write_bytes_per_sample': traffic.get('write_bytes_per_sample'), 'source': traffic['source']}
    vl = None
    if valu and valu.get('valu_insts_per_sample') and valu.get('clock_hz') and calib:
        clk = valu['clock_hz']
        cpi = calib['peak']['simd_cycles_per_wave_valu_inst']
        a = valu['valu_insts_per_sample'] * launch_samples / kernel_s / 1e9
        pk = 1024 * clk / cpi / 1e9
        busy = valu['valu_busy_cycles_per_sample'] * launch_samples / kernel_s / 1e9
        ia = valu['valu_insts_per_sample'] * 64 * launch_samples / kernel_s / 1e12
        ipk = 1024 * 32 * clk / 1e12
        vl = {'achieved': round(a, 2), 'peak': round(pk, 2), 'unit': 'G wave64 VALU instructions/s',
              'frac': round(a / pk, 5), 'valu_insts_per_sample': round(valu['valu_insts_per_sample'], 2),
              'calibration': {'simd_cycles_per_wave_valu_inst': cpi, 'source': calib['source'],
                              'kernel': calib['peak']['kernel'], 'busy_at_saturation': calib['peak']['valu_busy_per_simd']},
              'busy': {'achieved': round(busy, 1), 'peak': round(1024 * clk / 1e9, 1),
                       'unit': 'G VALU-busy SIMD-cycles/s', 'frac': round(busy / (1024 * clk / 1e9), 5)},
              'spec_lane_issue': {'achieved': round(ia, 3), 'peak': round(ipk, 3), 'unit': 'Tlane-op/s',
                                  'frac': round(ia / ipk, 5),
                                  'note': 'unpacked f32 VALU reaches at most ~0.48 of this (calibration)'},
              'clock_mhz': round(clk / 1e6, 1),
              'wait_frac_per_wave': round(valu['wait_frac_per_wave'], 4), 'source': valu['source']}
    cands = [(k, v) for k, v in (('hbm', hbm), ('valu', vl)) if v]
    reason = None
    if not cands:
        # no measured profile of this build: the model's bytes are no measurement, so no frac
        kind, top = 'hbm', dict(model, frac=None)
        reason = ('no rocprofv3 profile of this build (libmtsgpu.so sha256 %s): %s' % (
            (lib_hash or '?')[:12], '; '.join(stale) if stale else 'none committed'))
    else:
        kind, top = max(cands, key=lambda kv: kv[1]['frac'])
    line = {'bound': kind, 'achieved': top['achieved'], 'peak': top['peak'], 'unit': top['unit'], 'frac': top['frac'],
            'traffic': round(traffic['hbm_bytes_per_sample'] * launch_samples) if hbm else None,
            'traffic_unit': 'B per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, scaled to this launch)',
            'hbm': hbm, 'valu': vl, 'hbm_model': model, 'kernel_ms_avg': round(kernel_s * 1e3, 3),
            'lib_sha256': lib_hash}
    if stalls:
        line['stalls'] = {k: stalls.get(k) for k in ('per_sample', 'latency_cycles', 'source', 'lib_sha256')}
    if reason:
        line['frac_null_reason'] = reason
    elif stale:
        line['stale_profiles_ignored'] = stale
    return line


def host_info():
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, os.cpu_count() or 1, avail


def cgroup_cpus():
    """The job's cgroup CPU quota in CPUs (/sys/fs/cgroup/cpu.max: "quota period",
    or "max"), None when unlimited or unreadable."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        return None if q == 'max' else int(q) / int(per)
    except (OSError, ValueError):
        return None


def cpu_baseline(scene, integ, threads):
    """The CPU restatement (oracle, OpenMP, glibc transcendentals as the
    reference) on a bounded sample of the same workload: the full frame at a
    reduced spp (the first spp Sobol samples of every pixel, sized by two
    pilot passes to about 20 s of CPU work).  Threads: all
    cores this job may use -- OMP_NUM_THREADS when the host sets it (the GPU
    boxes give a job a 16-CPU share of a larger machine), else the affinity
    mask; never more than the cgroup's CPU quota, which the line records."""
    import copy
    import oracle.binding as ob
    model, ncpu, avail = host_info()
    quota = cgroup_cpus()
    omp = os.environ.get('OMP_NUM_THREADS')
    if not threads:
        threads = int(omp) if omp and omp.isdigit() and int(omp) > 0 else avail
        if quota:
            threads = max(1, min(threads, int(quota)))
    it = copy.copy(integ)
    # size the sample to ~20 s of CPU work: two pilot passes (1/8 of the rows
    # at 4 and 12 spp) give this config's marginal per-sample cost without the
    # per-render setup, then the full frame runs at the power-of-two spp
    # (1..256) nearest, in ratio, to the spp that fits
    def pilot(spp):
        it.sampleCount = spp
        t0 = time.perf_counter()
        _, _, pst = ob.render(scene, it, libm_mode=0, threads=threads, row=(1, 8, 0))
        return pst['samples'], time.perf_counter() - t0
    s1, t1 = pilot(4)
    s2, t2 = pilot(12)
    rate = (s2 - s1) / max(1e-6, t2 - t1) if t2 > t1 else s2 / max(1e-6, t2)
    fit = 20.0 * rate / (scene.sensor.width * scene.sensor.height)
    spp = 1
    cap = 256 if integ.rfilter == 'box' else 64   # gather mode keeps every sample's record (28 B) in host memory
    while spp * 2 <= min(integ.sampleCount, cap) and spp * 2 <= fit * 1.41421356:
        spp *= 2
    it.sampleCount = spp
    t0 = time.perf_counter()
    _, _, st = ob.render(scene, it, libm_mode=0, threads=threads)
    dt = time.perf_counter() - t0
    return {'value': round(st['samples'] / dt / 1e6, 3), 'unit': 'Msamples/s', 'cores': threads, 'kind': 'port',
            'sample': '%dx%d at %d spp (%d samples, %.1f s)' % (scene.sensor.width, scene.sensor.height,
                                                                it.sampleCount, st['samples'], dt),
            'cpu_model': model, 'host_cpus': ncpu, 'affinity_cpus': avail, 'omp_num_threads': omp,
            'cgroup_cpu_quota': quota}


def build_scene(config, size=None):
    sys.path.insert(0, REPO)
    from pkgimport import mitsuba_amd
    mitsuba_amd()
    from mitsuba_amd import scenes
    # C2g: C2 with Mitsuba's default reconstruction filter, gaussian stddev 0.5
    # (film.cpp:89-95, gaussian.cpp:35-56), the film gathered in a fixed order (film_gather)
    kw = {'rfilter': 'gaussian' if config.endswith('g') else 'box'}
    if size:
        w, h, spp = (int(v) for v in size.lower().split('x'))
        kw.update(width=w, height=h, spp=spp)
    return scenes.build(config[:-1] if config.endswith('g') else config, **kw)


def run_workload(config, args, world, rank, local, dist, torch, lib_hash):
    """Times args.steps frames of `config` (after args.warmup untimed ones) on
    this rank's tiles, bracketed by barrier + synchronize; returns rank 0's
    result dict (None on other ranks)."""
    scene, integ = build_scene(config, args.size)
    from mitsuba_amd import film_border
    from mitsuba_amd.distributed import TileSharding
    W, H, spp = scene.sensor.width, scene.sensor.height, integ.sampleCount
    b = film_border(integ.rfilter, integ.rfilterParam)
    shard = TileSharding.for_frame(rank, world, H)
    row = shard.row_params()
    gpu = args.device == 'gpu'

    if gpu:
        from mitsuba_amd.integrator import Context
        ctx = Context(torch.cuda.current_device())
        t_up = time.time()
        ctx.upload(scene)
        upload_s = time.time() - t_up
        film = torch.zeros(((H + 2 * b) * (W + 2 * b) * 5,), dtype=torch.float32, device='cuda')
        stream = torch.cuda.current_stream().cuda_stream
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(max(args.steps, 1))]

        def reduce():
            if args.share_device and world > 1:   # gloo: through host memory
                host = film.cpu()
                shard.reduce(host, dist)
                film.copy_(host)
            elif args.rccl and world == 1:        # the RCCL reduce of a one-rank job
                dist.reduce(film, dst=0, op=dist.ReduceOp.SUM)
            else:
                shard.reduce(film, dist)

        def step(k=None):   # mtsgpu_render_device clears the film on the stream
            st = ctx.render_device(integ, film.data_ptr(), stream, row=row, tile_shard=shard.tile_shard)
            if k is not None:
                ev[k][0].record()
            reduce()
            if k is not None:
                ev[k][1].record()
            return st

        def sync():
            torch.cuda.synchronize()
    else:
        import oracle.binding as ob
        upload_s = 0.0
        film = torch.zeros(((H + 2 * b) * (W + 2 * b) * 5,), dtype=torch.float32)
        threads = max(1, (os.cpu_count() or 1) // world)

        def step(k=None):
            f, _, st = ob.render(scene, integ, row=row, threads=threads, tile_shard=shard.tile_shard)
            film.copy_(torch.from_numpy(f.reshape(-1)))
            t = time.perf_counter()
            shard.reduce(film, dist)
            st['reduce_s'] = time.perf_counter() - t
            st['kernel_ms'] = 0.0
            return st

        def sync():
            pass

    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    kernel_ms, reduce_s = [], []
    samples_rank = 0
    for k in range(args.steps):
        st = step(k)
        kernel_ms.append(st['kernel_ms'])
        if 'reduce_s' in st:
            reduce_s.append(st['reduce_s'])
        samples_rank += st['samples']
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if gpu:
        reduce_s = [ev[k][0].elapsed_time(ev[k][1]) / 1e3 for k in range(args.steps)]
    dev = 'cuda' if gpu and not args.share_device else 'cpu'
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    s = torch.tensor([samples_rank], dtype=torch.float64, device=dev)
    r = torch.tensor([max(reduce_s) if reduce_s else 0.0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(r, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())
    total_samples = float(s.item())
    frame_samples = W * H * spp
    assert int(total_samples) == frame_samples * args.steps, (total_samples, frame_samples)
    if rank != 0:
        return None
    if args.save_film and config == args.config:
        import numpy as np
        np.save(args.save_film, film.cpu().numpy().reshape(H + 2 * b, W + 2 * b, 5))
    value = total_samples / elapsed_max / 1e6
    roofline = None
    cpu = None
    if gpu:
        # roofline: traversal counters from a bounded stats pass (1/16 of the rows), always
        # through the BVH: tiny scenes' linear TriAccel scan (an implementation choice that
        # reads every record from the scalar cache) must not inflate the workload's bytes
        os.environ['MTSGPU_NO_SCAN'] = '1'
        try:
            _, _, sst = ctx.render(integ, row=(8, 16, 0), traversal_stats=True)
        finally:
            os.environ.pop('MTSGPU_NO_SCAN', None)
        bps = algorithmic_bytes_per_sample(sst, scene.num_triangles, len(scene.emitters))
        avg_kernel_s = (sum(kernel_ms) / len(kernel_ms)) / 1e3
        per_launch_samples = samples_rank / max(1, len(kernel_ms))
        roofline = roofline_line(bps, per_launch_samples, avg_kernel_s, config, lib_hash)
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(scene, integ, args.cpu_threads)
    film_reduce = ('gloo' if args.share_device and world > 1 else
                   ('RCCL' if gpu and (world > 1 or args.rccl) else ('gloo' if world > 1 else 'none')))
    return {'value': round(value, 2), 'ms_per_step': round(elapsed_max / args.steps * 1e3, 2),
            'config': {'workload': WORKLOADS.get(config, config), 'width': W, 'height': H, 'spp': spp,
                       'samples_per_frame': frame_samples,
                       'parallelism': '8x8 tiles dealt over %d rank(s), film reduce: %s' % (world, film_reduce),
                       'world_size_reported': dist.get_world_size() if dist.is_initialized() else 1,
                       'reduce_ms_max': round(float(r.item()) * 1e3, 3),
                       's_per_frame': round(elapsed_max / args.steps, 4), 'scene_upload_s': round(upload_s, 3)},
            'roofline': roofline, 'cpu_baseline': cpu, 'spp': spp, 'W': W, 'H': H}


def main():
    args = parse_args()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)

    import torch  # loads the HIP runtime first; libmtsgpu shares it
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    gpu = args.device == 'gpu'
    lib_hash = None
    if gpu:
        if not torch.cuda.is_available():
            sys.exit('bench.py: no GPU visible (the HIP path has no CPU fallback; --device cpu-oracle is the '
                     'launcher rehearsal)')
        dev = 0 if args.share_device else local
        torch.cuda.set_device(dev)
        if world > 1 and args.share_device:
            dist.init_process_group('gloo')   # RCCL refuses two ranks on one device
        elif world > 1 or args.rccl:
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        lib_hash = lib_sha256()
    elif world > 1:
        dist.init_process_group('gloo')
    if world > 1:
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)

    main_res = run_workload(args.config, args, world, rank, local, dist, torch, lib_hash)
    second = {}
    if args.secondary and args.secondary.lower() != 'none' and not args.size:
        for cfg in [c.strip() for c in args.secondary.split(',') if c.strip()]:
            if cfg != args.config and cfg not in second:
                second[cfg] = run_workload(cfg, args, world, rank, local, dist, torch, lib_hash)

    if rank == 0:
        m = main_res
        metric = BASELINE_METRIC if args.config == 'C2' and not args.size else \
            'Msamples/s (and s/frame) at %d spp, %dx%d' % (m['spp'], m['W'], m['H'])
        out = {
            'metric': metric, 'value': m['value'],
            'unit': 'Msamples/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': m['ms_per_step'], 'higher_is_better': True,
            'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
            'config': m['config'],
            'roofline': m['roofline'],
            'cpu_baseline': m['cpu_baseline'],
        }
        if second:
            out['secondary'] = {cfg: {
                'metric': 'Msamples/s (and s/frame) at %d spp, %dx%d' % (r['spp'], r['W'], r['H']),
                'value': r['value'], 'unit': 'Msamples/s', 'ms_per_step': r['ms_per_step'],
                'steps': args.steps, 'warmup': args.warmup, 'config': r['config'],
                'roofline': r['roofline'], 'cpu_baseline': r['cpu_baseline']} for cfg, r in second.items()}
        if not gpu:
            out['device'] = 'cpu-oracle launcher rehearsal (not a GPU measurement)'
        elif args.share_device:
            out['device'] = 'shared-GPU rehearsal: %d ranks on GPU 0, gloo reduce (not a scaling measurement)' % world
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
