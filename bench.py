#!/usr/bin/env python3
"""bench.py -- device-resident RS(k,m) block erasure coding on MI355X.

Workload (BASELINE.json configs[1], "C2"): RS(10,4) encode of 4096 x 1 MiB
synthetic blocks per GPU, inputs resident in HBM before the timed region.
A "step" = one encode pass over the whole batch (one kernel launch).  With
--gpus N (torchrun, one process per GPU) every rank encodes its own 4096
blocks (block-index partition, BASELINE.json C4 at N=8): weak scaling, no
collective on the data path -- only the timing barrier / max-over-ranks.

Printed JSON line (rank 0): the contract fields plus
  roofline     : dominant kernel (gf_mac_kernel) algorithmic HBM bytes per
                 launch, (k+m)*S*n, / its average HIP-event duration, vs 8 TB/s
  cpu_baseline : the C oracle (scalar, table-driven) on this host's cores,
                 same workload bytes, bounded sample (rank 0, N=1 only)
  rebuild      : BASELINE.json C3 (RS(10,4), 4 random erasures per block)
  end_to_end   : pinned host -> HBM -> host rate (PCIe-inclusive; not `value`)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0x6D656D6F
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec, GB/s (MI355X_MICROARCH.md)
METRIC = "GiB/s RS(k,m) encode+rebuild, device-resident batched blocks; % HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # ~60 ms of back-to-back launches: the MI355X's clocks dip a few launches
    # into a burst and take ~40 launches to settle (profiles/r01_clock_ramp.jsonl)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--block-bytes", type=int, default=1 << 20)
    ap.add_argument("--blocks", type=int, default=4096, help="blocks per GPU")
    ap.add_argument("--erasures", type=int, default=4)
    ap.add_argument("--no-rebuild", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--sweep", action="store_true", help="also run the C5 mixed sweep")
    ap.add_argument("--sha", action="store_true",
                    help="also time GPU SHA-256 (CHB addresses) of the batch and of 4 KiB blocks")
    ap.add_argument("--sweep-gib", type=float, default=4.0, help="payload GiB per sweep point")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) or gloo (rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearse N>1 on a 1-GPU box with gloo)")
    return ap.parse_args()


def timed_launches(torch, fn, steps, warmup, dist, stream):
    """Warmup, then exactly `steps` launches bracketed by barrier+sync; per-
    launch HIP events on `stream` (the stream the kernels are enqueued on)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    kms = [a.elapsed_time(b) for a, b in ev]
    return wall, kms


def max_over_ranks(torch, dist, x):
    if dist is None:
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sweep(torch, ec, codec, stream, gib, steps, warmup):
    """BASELINE.json C5: (k,m) in {(4,2),(10,4),(16,4)} x B in 4 KiB..4 MiB,
    ~gib GiB of payload per point, one encode launch per step; then the same
    12 smaller groups as ONE memo_ec_encode_segments call (one launch per
    shard-chunk class, back to back; timed from before the first launch to
    after the last)."""
    points = []
    for (k, m) in [(4, 2), (10, 4), (16, 4)]:
        for B in [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20]:
            S = ec.shard_size(B, k)
            n = max(1, int(gib * 2**30) // B)
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            codec.fill_blocks(SEED, 0, n, B, k, S, d)
            _, kms = timed_launches(torch, lambda: codec.encode(k, m, d, p), steps, warmup, None, stream)
            ms = float(np.mean(kms))
            alg = (k + m) * S * n
            points.append({"k": k, "m": m, "block_bytes": B, "blocks": n, "shard_bytes": S,
                           "kernel_ms": round(ms, 4), "GiBs": round(n * B / (ms * 1e-3) / 2**30, 1),
                           "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)})
            del d, p
    segs, alg, pay = [], 0, 0
    for (k, m) in [(4, 2), (10, 4), (16, 4)]:
        for B in [4 << 10, 64 << 10, 1 << 20, 4 << 20]:
            S = ec.shard_size(B, k)
            n = max(1, int(gib * 2**30 / 12) // B)
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            codec.fill_blocks(SEED, 0, n, B, k, S, d)
            segs.append((k, m, S, n, d, p))
            alg += (k + m) * S * n
            pay += n * B
    _, kms = timed_launches(torch, lambda: codec.encode_segments(segs), steps, warmup, None, stream)
    ms = float(np.mean(kms))
    fused = {"segments": len(segs), "kernel_ms": round(ms, 4),
             "GiBs": round(pay / (ms * 1e-3) / 2**30, 1),
             "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    return {"workload": "BASELINE.json C5: RS(k,m) encode per (k,m) x block size, ~%.1f GiB "
                        "payload per point; fused = 12 mixed groups in one encode_segments call "
                        "(one launch per code class)" % gib,
            "points": points, "fused": fused}


def rebuild_small(torch, ec, codec, stream, steps, warmup):
    """Small-block rebuild: 4 KiB blocks (~4 GiB of payload), 4 random
    erasures per block, so every block has its own decode rows and a
    256-column tile spans up to 17 blocks' tables.  Step = decode + MAC."""
    res = {}
    for (k, m) in [(10, 4), (16, 4)]:
        B, n, e = 4096, 1 << 20, 4
        S = ec.shard_size(B, k)
        d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
        codec.fill_blocks(SEED, 0, n, B, k, S, d)
        codec.encode(k, m, d, p)
        s_idx, l_idx = ec.erasures(SEED, 0, n, k, m, e)
        sd, ld = torch.from_numpy(s_idx).cuda(), torch.from_numpy(l_idx).cuda()
        surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, d, p, sd, surv)
        want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, d, p, ld, want)
        del d, p
        out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        _, kms = timed_launches(torch, lambda: codec.rebuild(k, m, sd, surv, ld, out),
                                max(1, steps // 2), warmup, None, stream)
        codec.synchronize()
        ms = float(np.mean(kms))
        alg = (k + e) * S * n
        res["RS(%d,%d)" % (k, m)] = {
            "blocks": n, "block_bytes": B, "shard_bytes": S, "erasures": e,
            "step_ms": round(ms, 4), "GiBs": round(n * B / (ms * 1e-3) / 2**30, 1),
            "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "bit_exact": bool(torch.equal(out, want))}
        del surv, out, want, sd, ld
    return res


def _rate(fn, nbytes, seconds):
    """GiB/s of repeated fn() passes over ~`seconds` (at least one pass)."""
    passes, t = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t
        if el >= seconds:
            return passes * nbytes / el / 2**30, passes, el


def cpu_baseline(k, m, B, S, seconds, gpu_parity_sample):
    """Time the CPU codecs of oracle/ on this host, on a bounded sample of
    the same workload, and cross-check them against the GPU parity of the
    same blocks.  `value` is the vectorised encode (oracle/rs_simd.c:
    GFNI+AVX-512 affine or AVX2 split-nibble, ISA-L's published x86
    techniques), the strongest CPU codec here; the scalar table oracle is
    reported beside it.  Test infrastructure, never the product."""
    from oracle import oracle as O
    O.build()
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, 16))  # the GPU box's CPU share is 16 per GPU
    nb = 128
    data = O.aligned_empty((nb, k * S))
    data[:] = O.fill_blocks(SEED, 0, nb, B, k, S)
    par = O.aligned_empty((nb, m * S))
    nchk = gpu_parity_sample.shape[0]
    _, isa = O.encode_simd(k, m, S, data, threads=threads, out=par)
    ok_simd = bool(np.array_equal(par[:nchk], gpu_parity_sample))
    ok_scalar = bool(np.array_equal(O.encode(k, m, S, data[:nchk], threads=nchk), gpu_parity_sample))
    v, passes, el = _rate(lambda: O.encode_simd(k, m, S, data, threads=threads, isa=isa, out=par),
                          nb * B, seconds)
    one, _, _ = _rate(lambda: O.encode_simd(k, m, S, data[:64], threads=1, isa=isa, out=par[:64]),
                      64 * B, 1.5)
    sc_all, _, _ = _rate(lambda: O.encode(k, m, S, data[:32], threads=threads), 32 * B, 2.0)
    sc_one, _, _ = _rate(lambda: O.encode(k, m, S, data[:2], threads=1), 2 * B, 1.0)
    return {"value": round(v, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "RS(%d,%d) encode, %d x %d-byte blocks x %d passes (%.1f s), vectorised C port "
                      "(%s, streaming stores) on %d threads; 1-core %.3f GiB/s; scalar table oracle "
                      "%.3f GiB/s on %d threads, %.3f on 1; bit-exact vs GPU on %d blocks: %s"
                      % (k, m, nb, B, passes, el, O.SIMD_ISA[isa], threads, one, sc_all, threads,
                         sc_one, nchk, ok_simd and ok_scalar),
            "isa": O.SIMD_ISA[isa], "single_core": round(one, 3),
            "scalar_oracle": {"value": round(sc_all, 3), "single_core": round(sc_one, 3)},
            "bit_exact_vs_gpu": ok_simd and ok_scalar}


def c1_case(torch, ec, codec, stream):
    """BASELINE.json configs[0] (C1): RS(3,2) encode + rebuild (e = 1 and 2
    random erasures per block) of 1000 x 64 KiB blocks.  The CPU oracle
    (scalar, all host threads; the reference-runnable case) is timed beside
    the GPU on the same bytes, and every rebuilt shard is compared across
    the two (whole batch, bit-exact)."""
    from oracle import oracle as O
    k, m, B, n = 3, 2, 65536, 1000
    S = ec.shard_size(B, k)
    try:
        threads = max(1, min(len(os.sched_getaffinity(0)), 16))
    except AttributeError:
        threads = 1
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    t0 = time.perf_counter()
    par = O.encode(k, m, S, data, threads=threads)
    cpu_enc = time.perf_counter() - t0
    d = torch.from_numpy(data).cuda()
    p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    _, ek = timed_launches(torch, lambda: codec.encode(k, m, d, p), 20, 20, None, stream)
    ok = bool(np.array_equal(p.cpu().numpy(), par))
    out = {"workload": "RS(3,2) encode + rebuild (e=1, e=2), 1000 x 65536-byte blocks (BASELINE.json C1)",
           "cpu_threads": threads, "cpu_kind": "port (scalar table oracle)",
           "encode": {"cpu_ms": round(cpu_enc * 1e3, 3), "gpu_ms": round(float(np.median(ek)), 4)}}
    for e in (1, 2):
        s_idx, l_idx = O.erasures(SEED, 0, n, k, m, e)
        surv = O.gather(k, m, S, data, par, s_idx)
        t0 = time.perf_counter()
        want = O.rebuild(k, m, S, s_idx, surv, l_idx, threads=threads)
        cpu_reb = time.perf_counter() - t0
        sd, ld, sv = (torch.from_numpy(x).cuda() for x in (s_idx, l_idx, surv))
        o = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        _, rk = timed_launches(torch, lambda: codec.rebuild(k, m, sd, sv, ld, o), 20, 20, None, stream)
        codec.synchronize()
        ok = ok and bool(np.array_equal(o.cpu().numpy(), want))
        out["rebuild_e%d" % e] = {"cpu_ms": round(cpu_reb * 1e3, 3),
                                  "gpu_ms": round(float(np.median(rk)), 4)}
    out["bit_exact"] = ok
    return out


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if args.same_device:
        local = 0
    if world > 1:
        import torch.distributed as dist_mod
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist_mod.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist_mod.init_process_group(args.dist_backend)
        dist = dist_mod
    else:
        torch.cuda.set_device(0)
    from memo_amd import ec
    from memo_amd.partition import weak_range

    k, m, B, n, e = args.k, args.m, args.block_bytes, args.blocks, args.erasures
    S = ec.shard_size(B, k)
    # A dedicated (non-null) stream: the codec enqueues on it and the HIP
    # events that time each launch are recorded on the same stream.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    codec = ec.Codec(local if world > 1 else 0)
    codec.set_stream(stream)
    assert codec.stream == stream.cuda_stream and stream.cuda_stream

    data = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    first_block, _ = weak_range(n, rank)  # rank r owns blocks [r*n, (r+1)*n)
    codec.fill_blocks(SEED, first_block, n, B, k, S, data)
    torch.cuda.synchronize()

    enc = lambda: codec.encode(k, m, data, par)  # noqa: E731
    wall, kms = timed_launches(torch, enc, args.steps, args.warmup, dist, stream)
    codec.synchronize()
    wall = max_over_ranks(torch, dist, wall)
    kavg_ms = float(np.mean(kms))
    kavg_ms_max = max_over_ranks(torch, dist, kavg_ms)
    payload = world * n * B * args.steps
    value = payload / wall / 2**30
    alg_bytes = (k + m) * S * n
    achieved = alg_bytes / (kavg_ms * 1e-3) / 1e9

    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": "RS(%d,%d) encode, %d x %d-byte blocks per GPU (BASELINE.json %s)"
                               % (k, m, n, B, "C2" if world == 1 else "C4"),
                   "k": k, "m": m, "block_bytes": B, "blocks_per_gpu": n, "shard_bytes": S,
                   "global_blocks": n * world, "parallelism": "block-index partition x%d" % world},
        "roofline": {"bound": "hbm", "kernel": "gf_mac_kernel", "achieved": round(achieved, 1),
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                     "traffic": None, "bytes_per_launch": alg_bytes,
                     "kernel_ms_avg": round(kavg_ms, 4), "kernel_ms_min": round(min(kms), 4),
                     "kernel_ms_median": round(float(np.median(kms)), 4),
                     "kernel_ms_first_last": [round(kms[0], 4), round(kms[-1], 4)],
                     "kernel_ms_max_over_ranks": round(kavg_ms_max, 4),
                     "read_only_frac": round(k * S * n / (kavg_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)},
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            t = json.load(open(pmc))
            key = "encode_%d_%d_%d_%d" % (k, m, B, n)
            if key in t:
                result["roofline"]["traffic"] = t[key]["hbm_bytes_per_launch"]
                result["roofline"]["traffic_source"] = t[key]["source"]
        except Exception:
            pass

    # Measured HBM reference on this box: a device-to-device
    # copy of the same data bytes on the same stream (read + write).
    scratch = torch.empty_like(data)
    _, cms = timed_launches(torch, lambda: scratch.copy_(data), 10, 30, None, stream)
    copy_gbs = 2 * data.numel() / (float(np.median(cms)) * 1e-3) / 1e9
    result["roofline"]["copy_GBs"] = round(copy_gbs, 1)
    result["roofline"]["frac_of_copy"] = round(achieved / copy_gbs, 4)
    del scratch

    if not args.no_rebuild and e > 0:
        s_idx, l_idx = ec.erasures(SEED, first_block, n, k, m, e)
        sd = torch.from_numpy(s_idx).cuda()
        ld = torch.from_numpy(l_idx).cuda()
        surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, data, par, sd, surv)
        out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, data, par, ld, want)
        reb = lambda: codec.rebuild(k, m, sd, surv, ld, out)  # noqa: E731
        rwall, rkms = timed_launches(torch, reb, max(1, args.steps // 2), args.warmup, dist, stream)
        codec.synchronize()
        ok = bool(torch.equal(out, want))
        rwall = max_over_ranks(torch, dist, rwall)
        rsteps = max(1, args.steps // 2)
        rk = float(np.mean(rkms))
        rbytes = (k + e) * S * n
        result["rebuild"] = {
            "workload": "RS(%d,%d) rebuild, %d random erasures/block, %d x %d-byte blocks per GPU "
                        "(BASELINE.json C3)" % (k, m, e, n, B),
            "value": round(world * n * B * rsteps / rwall / 2**30, 3), "unit": "GiB/s",
            "ms_per_step": round(rwall / rsteps * 1e3, 4),
            "step_ms_events": round(rk, 4),
            "achieved_GBs": round(rbytes / (rk * 1e-3) / 1e9, 1),
            "frac": round(rbytes / (rk * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "note": "step = decode_coef_kernel (closed-form decode rows) + gf_mac_kernel",
            "round_trip_bit_exact": ok}
        del surv, out, want
        if world == 1:
            result["rebuild_small"] = rebuild_small(torch, ec, codec, stream, args.steps, args.warmup)

    if not args.no_e2e and world == 1:
        # PCIe-inclusive: blocks start and end in host memory (RPC socket in,
        # silos/peers out).  3-stage pipeline, 64 MiB batches; never `value`.
        ne = min(n, 1024)
        hd = torch.empty((ne, k * S), dtype=torch.uint8).pin_memory()
        hp = torch.empty((ne, m * S), dtype=torch.uint8).pin_memory()
        hd.copy_(data[:ne].cpu())
        codec.set_stream(None)
        e2e = {}
        for kind, (src, dst) in [("pinned", (hd, hp)),
                                 ("pageable", (hd.numpy().copy(), np.zeros((ne, m * S), np.uint8)))]:
            codec.encode(k, m, src, dst)
            t = time.perf_counter()
            reps = 6
            for _ in range(reps):
                codec.encode(k, m, src, dst)
            el = time.perf_counter() - t
            ok = bool(np.array_equal(np.asarray(dst[:4]), par[:4].cpu().numpy()))
            e2e[kind] = {"value": round(reps * ne * B / el / 2**30, 3), "bit_exact": ok}
        result["end_to_end"] = {
            "workload": "RS(%d,%d) encode, %d x %d-byte blocks from host memory, parity back to "
                        "host memory (HtoD + kernel + DtoH, 3-stage stream pipeline)" % (k, m, ne, B),
            "unit": "GiB/s", "pinned": e2e["pinned"], "pageable": e2e["pageable"]}
        # One-block host calls, as the plugin issues them for a lone store or
        # a degraded read (pageable elle::Buffer in, out): latency, not rate.
        lat = {}
        for bb in (4096, B):
            Sb = ec.shard_size(bb, k)
            d1 = np.frombuffer(np.random.default_rng(1).bytes(k * Sb), np.uint8).reshape(1, -1).copy()
            p1 = np.zeros((1, m * Sb), np.uint8)
            s1 = np.arange(1, k + 1, dtype=np.uint8).reshape(1, k)
            l1 = np.zeros((1, 1), np.uint8)
            o1 = np.zeros((1, Sb), np.uint8)
            for name, fn in (("encode", lambda: codec.encode(k, m, d1, p1)),
                             ("rebuild_e1", lambda: codec.rebuild(k, m, s1, d1, l1, o1))):
                for _ in range(20):
                    fn()
                ts = []
                for _ in range(200):
                    t = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - t)
                lat["%s_%dB_us" % (name, bb)] = round(float(np.median(ts)) * 1e6, 1)
        result["host_call_latency"] = dict(
            lat, note="median of 200 one-block calls from pageable host memory (copy in, kernels, "
                      "copy out, synchronous), RS(%d,%d)" % (k, m))
        codec.set_stream(stream)

    if rank == 0 and world == 1 and not args.no_cpu:
        sample = par[:4].cpu().numpy()
        result["cpu_baseline"] = cpu_baseline(k, m, B, S, args.cpu_seconds, sample)
        result["c1"] = c1_case(torch, ec, codec, stream)

    if args.sha and world == 1:
        import hashlib
        res = {}
        for name, nb, bb in [("C2 batch, 1 MiB blocks", n, B), ("4 KiB blocks", 1 << 20, 4096)]:
            msg = data if bb == B else torch.empty((nb, bb), dtype=torch.uint8, device="cuda")
            stride = msg.shape[1]
            if bb != B:
                codec.fill_blocks(SEED, 0, nb, bb, 1, bb, msg)
            pre = torch.zeros((nb, 64), dtype=torch.uint8, device="cuda")  # salt || owner
            dig = torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
            fn = lambda: codec.sha256(msg, dig, prefix=pre, uniform_len=bb, msg_stride=stride)  # noqa
            _, kms = timed_launches(torch, fn, 5, 1, None, stream)
            ms = float(np.mean(kms))
            ok = dig[0].cpu().numpy().tobytes() == hashlib.sha256(
                bytes(64) + msg[0, :bb].cpu().numpy().tobytes()).digest()
            one = msg[0, :bb].cpu().numpy().tobytes()
            t = time.perf_counter()
            reps = max(1, (64 << 20) // bb)
            for _ in range(reps):
                hashlib.sha256(one).digest()
            cpu = reps * bb / (time.perf_counter() - t) / 1e9
            res[name] = {"blocks": nb, "block_bytes": bb, "kernel_ms": round(ms, 3),
                         "GBs": round(nb * (bb + 64) / (ms * 1e-3) / 1e9, 1), "bit_exact": ok,
                         "cpu_1core_GBs": round(cpu, 2)}
            if bb != B:
                del msg
        result["sha256"] = {"workload": "batched SHA-256(salt||owner||data) = CHB addresses "
                                        "(CHB.cc:264-289), one lane per block", **res}

    if args.sweep and world == 1:
        del data, par
        result["sweep"] = sweep(torch, ec, codec, stream, args.sweep_gib, max(3, args.steps // 4), args.warmup)

    if rank == 0:
        print(json.dumps(result), flush=True)
    codec.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
