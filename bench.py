"""Headline benchmark: utterance-embeddings/sec (2 s @ 16 kHz), ERes2NetV2, fp32.

BASELINE.json configs[1]: ERes2NetV2 (17.8 M) batch=256 2 s segments, 1x MI355X fp32.
One step = the hot path over one batch of synthetic audio already resident in HBM:
GPU Kaldi Fbank (80 mel, mean-normalised) of 256 x 32000 samples -> ERes2NetV2 forward
-> 256 x 192 embeddings.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--with-allgather]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Multi-GPU: one process per GPU.  Under torch.distributed.run the ranks come from the
environment; a bare `bench.py --gpus N` (N > 1, no WORLD_SIZE) spawns the N rank processes
itself (spawn context, before this process touches the GPU), the way the reference's
infer_sv_batch.py:261-280 uses mp.spawn.  Utterances shard with no data-path collective
(weak scaling: every rank embeds its own 256-utterance batches); the barrier +
max-over-ranks timing is the only communication, unless --with-allgather adds the C4
exchange to every step (RCCL all-gather of the step's embeddings from every rank, then this
rank's row block of the cosine affinity consumed by the top-k kernel,
speakerlab/utils/distributed.py).  Rank 0 prints ONE JSON line, with the world size the
process group reports.  The roofline object describes the dominant
kernel (largest total time inside one forward), measured with HIP events on the stream
the kernels run on; the CPU baseline is the oracle (op-for-op torch CPU restatement)
timed on this host on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, '3d-speaker_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix (MFMA) peak
PEAK_FP16_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense FP16/BF16 MFMA peak (no sparsity)
# fp16x3 kernels (conv_gemm.hip): every fp32-accurate product costs three fp16 MFMA products,
# so their fp32-equivalent ceiling is the fp16 dense peak / 3
PEAK_X3_TFLOPS = PEAK_FP16_TFLOPS / 3
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec peak
BATCH = 256
SAMPLES = 32000               # 2 s @ 16 kHz -> 198 frames
METRIC = 'utterance-embeddings/sec (2 s @16 kHz)'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=BATCH)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-passes', type=int, default=5, help='timed CPU-baseline passes (best is reported)')
    ap.add_argument('--with-allgather', action='store_true',
                    help='add the C4 exchange (all-gather of the step embeddings + row-block top-1) to every step')
    ap.add_argument('--cpu-plumbing', action='store_true',
                    help='test mode without a GPU: gloo ranks, the step is the exchange on synthetic '
                         'embeddings only (exercises the launcher and the collectives, measures nothing)')
    ap.add_argument('--traffic-json', default=os.path.join(REPO, 'profiles', 'pmc_traffic.json'),
                    help='per-launch HBM bytes of the dominant kernel from a rocprofv3 --pmc pass (optional)')
    return ap.parse_args()


def build_model(device):
    from speakerlab.models.eres2net.ERes2NetV2 import ERes2NetV2
    from speakerlab.utils import synthetic
    bn_path = os.path.join(REPO, 'tests', 'golden', 'eres2netv2_bn.npz')
    bn = dict(np.load(bn_path)) if os.path.exists(bn_path) else None
    model = ERes2NetV2(feat_dim=80, embedding_size=192)
    synthetic.load_synthetic_weights(model, seed=0, bn_stats=bn)
    return model.eval().to(device)


def roofline(model, feats, device, traffic_json):
    """Per-step HIP-event timing of one forward; dominant kernel = largest total time."""
    h = model._hip_handle(device)
    B, T, _ = feats.shape
    plan = h.plan(B, T)
    out = torch.empty(B, 192, device=device)
    times = None
    for _ in range(3):                        # keep the last of 3 (warm)
        times = h.forward_timed(feats, out)
    nbytes = h.plan_bytes(B, T)
    groups = {}
    for (name, kern, fl), by, ms in zip(plan, nbytes, times):
        g = groups.setdefault(kern, {'ms': 0.0, 'flops': 0.0, 'bytes': 0.0, 'launches': 0, 'steps': []})
        g['ms'] += ms
        g['flops'] += fl
        g['bytes'] += by
        g['launches'] += 1
        g['steps'].append((fl, by, ms))
    kern, g = max(groups.items(), key=lambda kv: kv[1]['ms'])
    # fp16x3 kernels: the tiled / persistent x3 GEMMs and the fused Res2Net blocks
    x3 = '_x3' in kern or kern.startswith(('res2_block', 'aff_x3'))
    peak = PEAK_X3_TFLOPS if x3 else PEAK_FP32_TFLOPS

    def attainable(steps, pk):
        """Per-launch roofline: each launch needs at least max(FLOPs / MFMA peak, algorithmic
        bytes / HBM peak); summed over launches and compared with the measured time."""
        t_min = n_mfma = n_hbm = 0
        for fl, by, _ in steps:
            tf, tb = fl / (pk * 1e12), by / (PEAK_HBM_GBS * 1e9)
            t_min += max(tf, tb)
            n_mfma += tf >= tb
            n_hbm += tb > tf
        t = sum(ms for _, _, ms in steps) * 1e-3
        return {'attainable_ms': round(t_min * 1e3, 3), 'measured_ms': round(t * 1e3, 3),
                'frac': round(t_min / t, 4) if t else None,
                'launches_mfma_bound': int(n_mfma), 'launches_hbm_bound': int(n_hbm),
                'hbm_achieved_GBs': round(sum(by for _, by, _ in steps) / t / 1e9, 1) if t else None}
    avg_ms = g['ms'] / g['launches']
    flops_per_launch = g['flops'] / g['launches']
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12
    is_conv = lambda k: k.startswith(('conv_gemm', 'conv3x3', 'pw_gemm'))
    conv_ms = sum(v['ms'] for k, v in groups.items() if is_conv(k))
    conv_fl = sum(v['flops'] for k, v in groups.items() if is_conv(k))
    traffic = None
    if traffic_json and os.path.exists(traffic_json):
        try:
            t = json.load(open(traffic_json)).get(kern)
            traffic = None if t is None else round(t['bytes_per_launch'])
        except Exception:
            traffic = None
    # the kernel's binding roof: its launches' algorithmic bytes at 8 TB/s against their FLOPs
    # at the MFMA peak; the larger floor names the bound and the unit `achieved` is quoted in
    t_mfma = g['flops'] / (peak * 1e12)
    t_hbm = g['bytes'] / (PEAK_HBM_GBS * 1e9)
    hbm_bound = t_hbm > t_mfma
    bytes_per_launch = g['bytes'] / g['launches']
    gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    return {
        'kernel': kern,
        'bound': 'hbm' if hbm_bound else 'mfma',
        'achieved': round(gbs, 1) if hbm_bound else round(achieved, 3),
        'peak': PEAK_HBM_GBS if hbm_bound else round(peak, 1),
        'peak_basis': ('HBM3E 8 TB/s' if hbm_bound else
                       'fp16 dense MFMA 2500 TFLOP/s / 3 (fp16x3 split products, fp32-accurate)' if x3
                       else 'fp32 MFMA 157.3 TFLOP/s'),
        'unit': 'GB/s' if hbm_bound else 'TFLOP/s',
        'frac': round(gbs / PEAK_HBM_GBS, 4) if hbm_bound else round(achieved / peak, 4),
        'mfma_side': {'achieved_TFLOPs': round(achieved, 3), 'peak_TFLOPs': round(peak, 1),
                      'frac': round(achieved / peak, 4)},
        'hbm_side': {'achieved_GBs': round(gbs, 1), 'peak_GBs': PEAK_HBM_GBS, 'frac': round(gbs / PEAK_HBM_GBS, 4),
                     'algorithmic_bytes_per_launch': bytes_per_launch},
        'traffic': traffic,
        'traffic_unit': 'HBM bytes per launch (rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE, KiB -> B)',
        'launches_per_step': g['launches'],
        'avg_launch_ms': round(avg_ms, 4),
        'flops_per_launch': flops_per_launch,
        'all_conv_kernels': {'achieved': round(conv_fl / (conv_ms * 1e-3) / 1e12, 3),
                          'frac_of_x3_peak': round(conv_fl / (conv_ms * 1e-3) / 1e12 / PEAK_X3_TFLOPS, 4),
                          'ms_per_forward': round(conv_ms, 3)},
        'per_launch_roofline': dict(
            attainable(g['steps'], peak),
            basis='sum over the launches of max(algorithmic FLOPs / MFMA peak, algorithmic bytes / '
                  '8 TB/s) vs measured; bytes = every operand once (spk_model_plan_step_bytes)'),
        'all_conv_per_launch_roofline': attainable(
            [st for k, v in groups.items() if is_conv(k) for st in v['steps']], PEAK_X3_TFLOPS if x3 else peak),
        'forward_ms_sum_of_steps': round(sum(times), 3),
        'per_kernel_ms': {k: round(v['ms'], 3) for k, v in sorted(groups.items(), key=lambda kv: -kv[1]['ms'])},
    }


def fbank_roofline(wavs, device, reps=20):
    """The Fbank front end on its own: HIP events around `reps` back-to-back spk_fbank_f32
    calls (frames kernel + mean-normalisation kernel) on torch's current stream, the stream
    the library launches on.  Algorithmic bytes per utterance = 4 B per input sample + 4 B
    per output feature (every operand once)."""
    from speakerlab import _hip
    B, L = wavs.shape
    nfr = _hip.num_frames(L)
    offs = torch.tensor([[i * L for i in range(B + 1)], [i * nfr for i in range(B + 1)]],
                        dtype=torch.int64, device=device)
    feats = torch.empty(B * nfr, 80, device=device)
    lib, stream = _hip.lib(), torch.cuda.current_stream(device).cuda_stream

    def call():
        rc = lib.spk_fbank_f32(wavs.data_ptr(), offs[0].data_ptr(), B, feats.data_ptr(), offs[1].data_ptr(),
                               80, 1, stream)
        assert rc == 0, 'spk_fbank_f32 failed'
    for _ in range(3):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = B * (4 * L + 4 * 80 * nfr)
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {'kernel': 'fbank_frames_kernel + fbank_cmn_kernel', 'bound': 'hbm', 'achieved': round(gbs, 1),
            'peak': PEAK_HBM_GBS, 'unit': 'GB/s', 'frac': round(gbs / PEAK_HBM_GBS, 4),
            'avg_call_ms': round(ms, 4), 'bytes_per_call': nbytes,
            'basis': f'{B} utterances x ({4 * L} B samples in + {4 * 80 * nfr} B features out) per call, '
                     'HIP events over back-to-back calls'}


def physical_cores():
    """Physical cores of this host (lscpu: cores per socket x sockets), capped at the 16-CPU
    share a one-GPU box gives a job; os.cpu_count() counts SMT threads of the whole machine."""
    import subprocess
    try:
        out = subprocess.run(['lscpu'], capture_output=True, text=True, timeout=10).stdout
        info = {k.strip(): v.strip() for k, v in (l.split(':', 1) for l in out.splitlines() if ':' in l)}
        cores = int(info['Core(s) per socket']) * int(info.get('Socket(s)', '1'))
    except Exception:
        cores = os.cpu_count() or 1
    return max(1, min(16, cores))


def cpu_baseline(passes, batch=64):
    """Oracle (op-for-op torch CPU restatement + numpy Fbank) on the host cores, SURVEY §8(d):
    two warm-up passes, then the best of `passes` timed passes over one batch of `batch`
    utterances (a bounded sample of the C2 workload -- the first `batch` utterances of the
    batch the GPU leg times: a 256-utterance batch takes ~35 s per pass on 16 cores, so the
    sample is a quarter batch; ~60 s in all)."""
    from oracle import fbank_ref, models_ref
    from speakerlab.utils import synthetic
    from speakerlab.models.eres2net.ERes2NetV2 import ERes2NetV2
    threads = physical_cores()
    torch.set_num_threads(threads)
    bn = dict(np.load(os.path.join(REPO, 'tests', 'golden', 'eres2netv2_bn.npz')))
    sd = synthetic.load_synthetic_weights(ERes2NetV2(feat_dim=80, embedding_size=192), 0, bn).state_dict()
    # the first `batch` utterances of rank 0's timed C2 batch (run(): seed 1 + 1000 rank;
    # utterance i of a batch has its own seed, so this is a prefix of the same inputs)
    wavs = synthetic.pcm16_batch(batch, SAMPLES, seed=1)

    def one(w):
        feats = torch.from_numpy(fbank_ref.fbank_batch(w, 80, mean_nor=True))
        return models_ref.forward('eres2netv2', sd, feats)

    for _ in range(2):
        one(wavs)
    best = float('inf')
    for _ in range(passes):
        t0 = time.perf_counter()
        one(wavs)
        best = min(best, time.perf_counter() - t0)
    return {'value': round(batch / best, 3), 'unit': 'utt/s', 'cores': threads, 'kind': 'port',
            'sample': f'best of {passes} passes over the first {batch} utterances (2 s) of the timed C2 batch after 2 warm-up '
                      f'passes over the same batch; numpy Fbank + torch CPU fp32 oracle forward, {threads} physical cores '
                      f'(lscpu, capped at the box\'s 16-CPU share); best pass {best:.2f} s'}


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        return so.getsockname()[1]


def _rank_entry(rank, world, port, args):
    """Child process of the self-launcher: the torch.distributed.run environment, then run()."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    run(args)


def launch(args):
    """Spawn args.gpus rank processes (no GPU call in this parent: torch.cuda.device_count()
    does not initialise the runtime on this image); exit with the worst child status."""
    import torch.multiprocessing as mp
    n = args.gpus
    if not args.cpu_plumbing:
        have = torch.cuda.device_count()
        if have < n:
            raise SystemExit(f'bench.py --gpus {n}: only {have} GPU(s) visible')
    ctx = mp.get_context('spawn')
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(r, n, port, args)) for r in range(n)]
    for p in procs:
        p.start()
    for p in procs:
        p.join()
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad:
        raise SystemExit(f'bench.py: rank process(es) failed with exit codes {bad}')


def exchange_fn(emb, world, rank, n_total):
    """C4 exchange on the step's embeddings: the all-gather of every rank's [B, E] block (RCCL
    all_gather_into_tensor under nccl), then this rank's row block consumed by the top-1
    cosine kernel (self excluded)."""
    import torch.distributed as tdist
    from speakerlab.utils.distributed import all_gather_embeddings, topk_row_block
    emb_all = all_gather_embeddings(emb, n_total) if tdist.is_initialized() else emb
    if emb.is_cuda:
        return topk_row_block(emb_all, rank, world, k=1)
    return emb_all


def plumbing(args, world, rank):
    """--cpu-plumbing: the launcher + process group + exchange without a GPU (gloo)."""
    import torch.distributed as tdist
    B, E = 8, 192
    g = torch.Generator().manual_seed(rank)
    emb = torch.randn(B, E, generator=g)
    for _ in range(args.warmup):
        exchange_fn(emb, world, rank, B * world)
    if world > 1:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = exchange_fn(emb, world, rank, B * world)
    if world > 1:
        tdist.barrier()
    dt = time.perf_counter() - t0
    ok = got.shape == (B * world, E) and torch.equal(got[rank * B:(rank + 1) * B], emb)
    t = torch.tensor([dt])
    if world > 1:
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item()), B, bool(ok)


def run(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = world > 1
    tdist = None
    if dist:
        import torch.distributed as tdist
        if args.cpu_plumbing:
            tdist.init_process_group('gloo')
        else:
            dev = torch.device('cuda', local)
            torch.cuda.set_device(dev)
            tdist.init_process_group('nccl', device_id=dev)
        world = tdist.get_world_size()
    if args.gpus != world and rank == 0:
        print(f'bench.py: --gpus {args.gpus} but the process group has {world} rank(s); '
              f'reporting n_gpus = {world}', file=sys.stderr, flush=True)

    if args.cpu_plumbing:
        dt, B, ok = plumbing(args, world, rank)
        if rank == 0:
            print(json.dumps({'metric': METRIC + ' [cpu plumbing test: no GPU work]', 'value': None,
                              'n_gpus': world, 'world_size': world, 'backend': tdist.get_backend() if dist else None,
                              'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(dt / args.steps * 1e3, 3),
                              'exchange_ok': ok, 'rows_per_rank': B}), flush=True)
        if dist:
            tdist.destroy_process_group()
        return

    device = torch.device('cuda', local)
    torch.cuda.set_device(device)

    from speakerlab import _hip
    from speakerlab.utils import synthetic

    model = build_model(device)
    B = args.batch
    wavs = torch.from_numpy(synthetic.pcm16_batch(B, SAMPLES, seed=1 + 1000 * rank)).to(device)

    def step():
        feats = _hip.fbank(wavs, 80, mean_nor=True)
        emb = model(feats)
        if args.with_allgather:
            exchange_fn(emb, world, rank, B * world)
        return emb

    handle = model._hip_handle(device)
    reruns, checked = 0, 0                    # fp16x3 range guard: forwards the exact plan re-ran
    with torch.no_grad():
        for _ in range(args.warmup):
            step()
            reruns += int(handle.last_forward_exact)   # untimed: checked after every warm-up forward
            checked += 1
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            emb = step()
        torch.cuda.synchronize()
        if dist:
            tdist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert torch.isfinite(emb).all(), 'non-finite embeddings'
        reruns += int(handle.last_forward_exact)       # the last timed forward (same input every step)
        checked += 1
        if dist:
            t = torch.tensor([dt], device=device)
            tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
            dt = float(t.item())
        exchange = None
        if args.with_allgather:
            # the exchange alone, HIP events on torch's stream (RCCL and the top-k kernel run there)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                exchange_fn(emb, world, rank, B * world)
            e1.record()
            e1.synchronize()
            exchange = {'ms_per_step': round(e0.elapsed_time(e1) / reps, 4), 'rows_gathered': B * world,
                        'allgather_bytes': 4 * 192 * B * world,
                        'what': 'all_gather_embeddings (RCCL) + topk_row_block (spk_cosine_topk, k=1), rank 0'}
        feats = _hip.fbank(wavs, 80, mean_nor=True)
        roof = roofline(model, feats, device, args.traffic_json) if rank == 0 else None
        if roof is not None:
            roof['fbank'] = fbank_roofline(wavs, device)

    total_utts = B * args.steps * world
    value = total_utts / dt
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.cpu_passes)
        flops = model._hip_handle(device).flops(198)
        line = {
            'metric': METRIC,
            'value': round(value, 2),
            'unit': 'utt/s',
            'n_gpus': world,
            'world_size': world,
            'backend': tdist.get_backend() if dist else None,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(dt / args.steps * 1e3, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f32 (fp16x3 split-precision MFMA, fp32 accumulate)',
            'data': 'synthetic PCM16 speech-like audio (numpy PCG64), deterministic synthetic weights',
            'config': {'workload': 'ERes2NetV2 (17.8 M) batch=256 2 s segments, GPU Fbank + embedding, fp32'
                                   + (' + C4 exchange per step' if args.with_allgather else ''),
                       'model': 'ERes2NetV2', 'global_batch': B * world, 'seq_len': 198,
                       'parallelism': f'dp{world} (utterance sharding, '
                                      + ('RCCL all-gather of the embeddings per step)' if args.with_allgather
                                         else 'no data-path collective)')},
            'model_tflops_achieved': round(value * flops / 1e12, 3),
            'model_gflop_per_utt': round(flops / 1e9, 3),
            'exchange': exchange,
            # the range guard's exact-fp32 re-run must never fire on this input
            'exact_reruns': {'count': reruns, 'forwards_checked': checked},
            'roofline': roof,
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        launch(args)
    else:
        run(args)


if __name__ == '__main__':
    main()
