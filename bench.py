#!/usr/bin/env python3
"""bench.py -- device-resident RS(k,m) block erasure coding on MI355X.

Metric (BASELINE.json): GiB/s of RS(k,m) encode+rebuild over device-resident
batched blocks, with the kernels' fraction of the HBM roofline.

A "step" is one pass of the hot path over the batch in both directions:
  * encode  -- BASELINE.json configs[1] (C2): RS(10,4) parity of 4096 x 1 MiB
               synthetic blocks (one gf_mac_kernel launch);
  * rebuild -- configs[2] (C3): the same 4096 blocks rebuilt from k of their
               k+m shards with 4 random shards lost per block
               (decode_coef_kernel rows, then gf_mac_kernel).
Inputs are resident in HBM before the timed region.  `value` = payload bytes
encoded + payload bytes rebuilt, over all ranks, / the job's wall time.

--gpus N: one process per GPU.  Without an external launcher (WORLD_SIZE
unset) bench.py starts the N ranks itself before touching any GPU; under
torch.distributed.run it uses the launcher's ranks.  Every rank encodes and
rebuilds its own 4096 blocks (block-index partition; BASELINE.json C4 at N=8):
weak scaling.  The barrier and the max-over-ranks run over gloo on the host;
nothing crosses GPUs (no RCCL).

Printed JSON line (rank 0): the contract fields plus
  encode / rebuild : per-direction GiB/s, kernel ms and roofline fraction
  roofline         : the encode kernel (C2, the north-star target): its
                     algorithmic bytes per launch (k+m)*S*n / its average
                     HIP-event duration, vs 8 TB/s; roofline_rebuild likewise;
                     `traffic` from rocprofv3 counter passes this run makes
                     (pmc_traffic)
  ranks            : per-GPU GiB/s, node sum (C4's wording)
  cpu_baseline     : the C port (oracle/, test infrastructure) timed on this
                     host's CPU share on a bounded sample (rank 0, every N,
                     after the timed steps)
  end_to_end       : pinned host -> HBM -> host rate (PCIe-inclusive; not
                     `value`), every rank over its own link, node sum at N>1
  build_id         : memo_ec_build_id() of the loaded library (== SHA-256 of
                     the sources in this tree: build_matches_sources)
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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--warmup", type=int, default=30)
    # The MI355X's clocks dip a few launches into a burst and take ~40 ms of
    # back-to-back launches to settle (profiles/r01_clock_ramp.jsonl): untimed
    # steps continue past --warmup until this much wall time has gone by.
    ap.add_argument("--settle-ms", type=float, default=150.0)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--block-bytes", type=int, default=1 << 20)
    ap.add_argument("--blocks", type=int, default=4096, help="blocks per GPU")
    ap.add_argument("--erasures", type=int, default=4)
    ap.add_argument("--no-small", action="store_true", help="skip the 4 KiB random-rebuild lines")
    ap.add_argument("--small-only", action="store_true",
                    help=argparse.SUPPRESS)  # the counter pass child of pmc_small: 4 KiB lines only
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 FETCH_SIZE / WRITE_SIZE passes behind roofline.traffic")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--sweep", action="store_true", help="also run the C5 mixed sweep")
    ap.add_argument("--no-sha", action="store_true",
                    help="skip the GPU SHA-256 (CHB address) lines over the batch and 1M x 4 KiB blocks")
    ap.add_argument("--sweep-gib", type=float, default=4.0, help="payload GiB per sweep point")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearse N>1 on a 1-GPU box)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the whole-batch oracle comparisons after the timed steps")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 mixed-geometry point")
    ap.add_argument("--c5-gib", type=float, default=4.0, help="payload GiB of the C5 mixed point")
    ap.add_argument("--no-plugin", action="store_true",
                    help="skip the plugin-level lines (host/_build/bench_plugin child runs)")
    ap.add_argument("--rank-timeout", type=float, default=600.0,
                    help="seconds a rank may take (launcher kill bound, gloo collective timeout)")
    return ap.parse_args(argv)


def log(msg):
    """Progress on stderr (stdout carries only the JSON line): long runs keep
    showing signs of life."""
    # one write per line: ranks share the stream, and print() writes the
    # text and the newline separately
    sys.stderr.write("[bench %.1fs] %s\n" % (time.perf_counter() - _T0, msg))
    sys.stderr.flush()


_T0 = time.perf_counter()


def timed_steps(torch, fns, steps, warmup, settle_ms, dist, stream):
    """`warmup` untimed steps (continued until settle_ms of wall time has gone
    by), then exactly `steps` steps bracketed by barrier + synchronize.  A
    step runs fns in order; HIP events on `stream` (the stream the kernels
    are enqueued on) bracket each fn.  Returns (wall seconds, per-fn lists of
    per-step ms, untimed steps run)."""
    t0 = time.perf_counter()
    done = 0
    while done < warmup or (time.perf_counter() - t0) * 1e3 < settle_ms:
        for f in fns:
            f()
        done += 1
        if done % 8 == 0:
            torch.cuda.synchronize()  # keep the host from queueing far ahead
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(len(fns) + 1)] for _ in range(steps)]
    t = time.perf_counter()
    for es in ev:
        es[0].record(stream)
        for f, e in zip(fns, es[1:]):
            f()
            e.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t
    ms = [[es[i].elapsed_time(es[i + 1]) for es in ev] for i in range(len(fns))]
    return wall, ms, done


def kstats(kms, alg_bytes):
    """Kernel-time summary of one direction: HIP-event ms per launch and the
    algorithmic-byte roofline fraction of the average launch."""
    avg = float(np.mean(kms))
    achieved = alg_bytes / (avg * 1e-3) / 1e9
    return {"kernel_ms_avg": round(avg, 4), "kernel_ms_min": round(min(kms), 4),
            "kernel_ms_median": round(float(np.median(kms)), 4),
            "kernel_ms_first_last": [round(kms[0], 4), round(kms[-1], 4)],
            "achieved": round(achieved, 1), "frac": round(achieved / PEAK_HBM_GBS, 4)}


def sweep(torch, ec, codec, stream, gib, steps, warmup, settle_ms, cpu=True):
    """BASELINE.json C5: (k,m) in {(4,2),(10,4),(16,4)} x B in 4 KiB..4 MiB,
    ~gib GiB of payload per point.  Each point times one encode launch and
    one rebuild of the same blocks with e = m random erasures per block (the
    metric is encode+rebuild), both checked bit-exact on the GPU.  Then the
    12-group mixed calls of c5_mixed."""
    def frac(alg, ms):
        return round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)

    def rebuild_inputs(k, m, S, n, d, p, fb=0):
        e = m
        s_idx, l_idx = ec.erasures(SEED, fb, n, k, m, e)
        sd, ld = torch.from_numpy(s_idx).cuda(), torch.from_numpy(l_idx).cuda()
        surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, d, p, sd, surv)
        want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, d, p, ld, want)
        out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        return e, s_idx, l_idx, sd, ld, surv, want, out

    points = []
    for (k, m) in [(4, 2), (10, 4), (16, 4)]:
        for B in [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20]:
            S = ec.shard_size(B, k)
            n = max(1, int(gib * 2**30) // B)
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            codec.fill_blocks(SEED, 0, n, B, k, S, d)
            codec.encode(k, m, d, p)
            e, s_idx, l_idx, sd, ld, surv, want, out = rebuild_inputs(k, m, S, n, d, p)
            _, (kms, rms), _ = timed_steps(
                torch, [lambda: codec.encode(k, m, d, p), lambda: codec.rebuild(k, m, sd, surv, ld, out)],
                steps, warmup, settle_ms, None, stream)
            codec.synchronize()
            ms, rs = float(np.mean(kms)), float(np.mean(rms))
            pt = {"k": k, "m": m, "block_bytes": B, "blocks": n, "shard_bytes": S,
                  "kernel_ms": round(ms, 4), "GiBs": round(n * B / (ms * 1e-3) / 2**30, 1),
                  "frac": frac((k + m) * S * n, ms),
                  "rebuild": {"erasures": e, "kernel": codec.rebuild_path(n, k, S, e), "step_ms": round(rs, 4),
                              "GiBs": round(n * B / (rs * 1e-3) / 2**30, 1),
                              "frac": frac((k + e) * S * n, rs),
                              "bit_exact": bool(torch.equal(out, want))},
                  "encode_rebuild_GiBs": round(2 * n * B / ((ms + rs) * 1e-3) / 2**30, 1)}
            if cpu:
                # CPU baseline of the point (per C5 point): the
                # vectorised port on 16 threads over a ~64 MiB sample of the
                # blocks, encode and the same blocks' rebuild
                from oracle import oracle as O
                nc = max(16, min(n, (64 << 20) // B))
                hd = O.aligned_empty((nc, k * S))
                hd[:] = d[:nc].cpu().numpy()
                hp = O.aligned_empty((nc, m * S))
                th = cpu_threads()
                _, isa = O.encode_simd(k, m, S, hd, threads=th, out=hp)
                ok = bool(np.array_equal(hp, p[:nc].cpu().numpy()))
                cv, _, _ = _rate(lambda: O.encode_simd(k, m, S, hd, threads=th, isa=isa, out=hp),
                                 nc * B, 0.4)
                hs = O.gather(k, m, S, hd, hp, s_idx[:nc])
                ho = O.aligned_empty((nc, e * S))
                O.rebuild_simd(k, m, S, s_idx[:nc], hs, l_idx[:nc], threads=th, isa=isa, out=ho)
                ok = ok and bool(np.array_equal(ho, out[:nc].cpu().numpy()))
                rv, _, _ = _rate(lambda: O.rebuild_simd(k, m, S, s_idx[:nc], hs, l_idx[:nc], threads=th,
                                                        isa=isa, out=ho), nc * B, 0.4)
                pt["cpu_GiBs"] = round(cv, 2)
                pt["cpu_rebuild_GiBs"] = round(rv, 2)
                pt["cpu_threads"] = th
                pt["cpu_bit_exact"] = ok
            points.append(pt)
            log("sweep RS(%d,%d) %d B: encode %.3f, rebuild %.3f" % (k, m, B, pt["frac"], pt["rebuild"]["frac"]))
            del d, p, surv, want, out, sd, ld
    fused = c5_mixed(torch, ec, codec, stream, gib, steps, warmup, settle_ms)
    return {"workload": "BASELINE.json C5: RS(k,m) encode and rebuild (e = m random erasures per "
                        "block) per (k,m) x block size, ~%.1f GiB payload per point; fused = 12 "
                        "mixed groups in one encode_segments call and one rebuild_segments call "
                        "(one launch per code class)" % gib,
            "points": points, "fused": fused}


def rebuild_small(torch, ec, codec, stream, steps, warmup, settle_ms, stage=None, threads=1,
                  uniform=True):
    """Small-block rebuild: 4 KiB blocks (~4 GiB of payload), 4 random
    erasures per block, so every block has its own decode rows and a
    256-column tile spans up to 17 blocks.  Encode of the same blocks is
    timed beside it (same process, same clocks), and so is the repair case
    of one pattern for every block (memo_ec_rebuild_uniform).  The memory
    system's rate for the same traffic (memo_ec_stream_probe) is the
    achievable denominator.  With a HostStage, the whole per-block-pattern
    batch is compared with the CPU oracle's rebuild, and the uniform one
    with the original shards."""
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
        out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        _, (ekms, rkms), _ = timed_steps(
            torch, [lambda: codec.encode(k, m, d, p), lambda: codec.rebuild(k, m, sd, surv, ld, out)],
            steps, warmup, settle_ms, None, stream)
        codec.synchronize()
        ms = float(np.mean(rkms))
        alg = (k + e) * S * n
        ok = bool(torch.equal(out, want))
        probe = probe_rate(torch, codec, stream, k, e, surv, want)
        codec.gather_shards(k, m, S, n, d, p, ld, want)  # the probe overwrote it
        row = {"blocks": n, "block_bytes": B, "shard_bytes": S, "erasures": e,
               "kernel": codec.rebuild_kernel_name(n, k, S),
               "step_ms": round(ms, 4), "GiBs": round(n * B / (ms * 1e-3) / 2**30, 1),
               "frac": round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
               "encode_frac_same_blocks": round((k + m) * S * n / (float(np.mean(ekms)) * 1e-3) / 1e9
                                                / PEAK_HBM_GBS, 4),
               "achievable": probe, "frac_of_achievable": round(probe["kernel_ms_avg"] / ms, 4),
               "bit_exact": ok}
        if stage is not None:
            row["oracle"] = verify_rebuild(stage, k, m, S, s_idx, surv, l_idx, out, threads)
        res["RS(%d,%d)" % (k, m)] = row
        if not uniform:
            del d, p, surv, out, want, sd, ld
            continue
        # the repair case: one lost node, every block the same pattern
        # (memo_ec_rebuild_uniform), here block 0's
        su, lu = s_idx[0], l_idx[0]
        sdu = torch.from_numpy(np.ascontiguousarray(np.tile(su, (n, 1)))).cuda()
        ldu = torch.from_numpy(np.ascontiguousarray(np.tile(lu, (n, 1)))).cuda()
        codec.gather_shards(k, m, S, n, d, p, sdu, surv)
        codec.gather_shards(k, m, S, n, d, p, ldu, want)
        _, (ukms,), _ = timed_steps(torch, [lambda: codec.rebuild_uniform(k, m, su, surv, lu, out)],
                                    steps, warmup, settle_ms, None, stream)
        codec.synchronize()
        ums = float(np.mean(ukms))
        row["uniform_pattern"] = {"step_ms": round(ums, 4),
                                  "frac": round(alg / (ums * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                                  "bit_exact": bool(torch.equal(out, want)),
                                  "check": "every rebuilt shard == the original shard it replaces"}
        log("rebuild_small RS(%d,%d): %.3f of peak, %.3f of achievable" % (
            k, m, row["frac"], row["frac_of_achievable"]))
        del d, p, surv, out, want, sd, ld, sdu, ldu
    return res


C5_CODES = [(4, 2), (10, 4), (16, 4)]
C5_SIZES = [4 << 10, 64 << 10, 1 << 20, 4 << 20]


def side_stream_decodes(ec, codec):
    """The ctx's MEMO_EC_OPT_DECODE_OVERLAP (None: a library without it)."""
    try:
        return bool(codec.get_option("decode_overlap"))
    except (ec.MemoECError, KeyError):
        return None


def c5_mixed(torch, ec, codec, stream, gib, steps, warmup, settle_ms, stage=None, threads=1):
    """BASELINE.json C5 as the plugin issues it: 12 groups, (k,m) in
    {(4,2),(10,4),(16,4)} x B in {4 KiB, 64 KiB, 1 MiB, 4 MiB}, ~gib GiB of
    payload in all, encoded by ONE memo_ec_encode_segments call and rebuilt
    (e = m random erasures per block) by ONE memo_ec_rebuild_segments call --
    the shape of a multi-address fetch, which hands a whole mixed batch to one
    call (Consensus::_fetch(vector<AddressVersion>), src/memo/model/doughnut/
    Consensus.cc:101-124; Paxos::_fetch, consensus/Paxos.cc:1857-1890).  One
    launch per code class, back to back; timed from before the first launch
    to after the last.  With a HostStage every group's parity and rebuilt
    shards are compared with the CPU oracle, and the rebuilt shards with the
    original ones."""
    def frac(alg, ms):
        return round(alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)

    groups, segs, rsegs, alg, ralg, pay = [], [], [], 0, 0, 0
    for gi, (k, m) in enumerate(C5_CODES):
        for B in C5_SIZES:
            S = ec.shard_size(B, k)
            n = max(1, int(gib * 2**30 / (len(C5_CODES) * len(C5_SIZES))) // B)
            e = m
            d = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
            codec.fill_blocks(SEED, 0, n, B, k, S, d)
            s_idx, l_idx = ec.erasures(SEED, gi, n, k, m, e)
            sd, ld = torch.from_numpy(s_idx).cuda(), torch.from_numpy(l_idx).cuda()
            surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
            want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
            out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
            groups.append(dict(k=k, m=m, B=B, S=S, n=n, e=e, d=d, p=p, s_idx=s_idx, l_idx=l_idx,
                               sd=sd, ld=ld, surv=surv, want=want, out=out))
            segs.append((k, m, S, n, d, p))
            rsegs.append(dict(k=k, m=m, surv_idx=sd, surv=surv, lost_idx=ld, out=out))
            alg += (k + m) * S * n
            ralg += (k + e) * S * n
            pay += n * B
    # parity by the mixed call itself, then the survivors / lost shards of it
    codec.encode_segments(segs)
    for g in groups:
        codec.gather_shards(g["k"], g["m"], g["S"], g["n"], g["d"], g["p"], g["sd"], g["surv"])
        codec.gather_shards(g["k"], g["m"], g["S"], g["n"], g["d"], g["p"], g["ld"], g["want"])
    _, (kms, rms), _ = timed_steps(torch, [lambda: codec.encode_segments(segs),
                                           lambda: codec.rebuild_segments(rsegs)],
                                   steps, warmup, settle_ms, None, stream)
    codec.synchronize()
    ms, rs = float(np.mean(kms)), float(np.mean(rms))
    res = {"workload": "BASELINE.json C5: 12 groups (k,m) in {(4,2),(10,4),(16,4)} x B in {4 KiB, "
                       "64 KiB, 1 MiB, 4 MiB}, %.1f GiB payload; one encode_segments call and one "
                       "rebuild_segments call (e = m random erasures per block) per step" % (pay / 2**30),
           "segments": len(segs), "payload_bytes": pay,
           "encode": {"kernel_ms": round(ms, 4), "GiBs": round(pay / (ms * 1e-3) / 2**30, 1),
                      "frac": frac(alg, ms), "bytes_per_call": alg},
           "rebuild": {"step_ms": round(rs, 4), "GiBs": round(pay / (rs * 1e-3) / 2**30, 1),
                       "frac": frac(ralg, rs), "bytes_per_call": ralg,
                       "side_stream_decodes": side_stream_decodes(ec, codec)},
           "encode_rebuild_GiBs": round(2 * pay / ((ms + rs) * 1e-3) / 2**30, 1)}
    per = []
    for g in groups:
        x = {"k": g["k"], "m": g["m"], "block_bytes": g["B"], "blocks": g["n"],
             "round_trip_bit_exact": bool(torch.equal(g["out"], g["want"]))}
        if stage is not None:
            ve = verify_encode(stage, g["k"], g["m"], g["S"], g["d"], g["p"], threads)
            vr = verify_rebuild(stage, g["k"], g["m"], g["S"], g["s_idx"], g["surv"], g["l_idx"],
                                g["out"], threads)
            x["oracle_encode_bit_exact"] = ve["bit_exact"]
            x["oracle_rebuild_bit_exact"] = vr["bit_exact"]
        per.append(x)
    res["groups"] = per
    res["round_trip_bit_exact"] = all(x["round_trip_bit_exact"] for x in per)
    if stage is not None:
        res["oracle_bit_exact"] = all(x["oracle_encode_bit_exact"] and x["oracle_rebuild_bit_exact"]
                                      for x in per)
    log("c5 mixed: encode %.3f, rebuild %.3f of peak" % (res["encode"]["frac"], res["rebuild"]["frac"]))
    return res


class HostStage:
    """Page-locked host staging for the whole-batch oracle comparisons:
    device rows are copied chunk by chunk (one DMA each, ~chunk_bytes per
    buffer) into reused pinned buffers, the CPU oracle runs on them, and no
    batch is ever held whole in host memory (an 8-rank node checks 8
    batches at once)."""

    def __init__(self, torch, chunk_bytes=256 << 20):
        self.torch = torch
        self.chunk = chunk_bytes
        self.pinned = {}
        self.plain = {}

    def rows_per_chunk(self, row_bytes):
        return max(1, self.chunk // row_bytes)

    def fetch(self, name, dev, r0, r1):
        """numpy view of rows [r0, r1) of a 2-D uint8 device tensor."""
        t = self.torch
        cols = dev.shape[1]
        nb = (r1 - r0) * cols
        b = self.pinned.get(name)
        if b is None or b.numel() < nb:
            b = t.empty(max(nb, self.chunk), dtype=t.uint8, pin_memory=t.cuda.is_available())
            self.pinned[name] = b
        v = b[:nb].view(r1 - r0, cols)
        v.copy_(dev[r0:r1])
        return v.numpy()

    def scratch(self, name, rows, cols):
        """64-byte-aligned host rows (the oracle's output)."""
        from oracle import oracle as O
        nb = rows * cols
        b = self.plain.get(name)
        if b is None or b.size < nb:
            b = O.aligned_empty((max(nb, self.chunk),))
            self.plain[name] = b
        return b[:nb].reshape(rows, cols)


def same_bytes(a, b):
    """a == b over two equal-shape uint8 arrays, in 64 MiB slices (no
    full-size boolean temporary)."""
    if a.shape != b.shape:
        return False
    x, y = a.reshape(-1), b.reshape(-1)
    step = 64 << 20
    return all(np.array_equal(x[i:i + step], y[i:i + step]) for i in range(0, x.size, step))


def verify_encode(stage, k, m, S, d, p, threads):
    """Every parity byte of a device batch against the CPU oracle
    (oracle/rs_simd.c, itself checked against the scalar oracle and the
    golden fixtures by tests/test_oracle.py) run on the same data bytes."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    n = d.shape[0]
    step = stage.rows_per_chunk((k + m) * S)
    ok = True
    for r0 in range(0, n, step):
        r1 = min(n, r0 + step)
        hd = stage.fetch("in", d, r0, r1)
        hp = stage.fetch("out", p, r0, r1)
        want = stage.scratch("want", r1 - r0, m * S)
        O.encode_simd(k, m, S, hd, threads=threads, out=want)
        ok = ok and same_bytes(want, hp)
    return {"blocks": n, "bytes_compared": n * m * S, "bit_exact": ok,
            "seconds": round(time.perf_counter() - t0, 2)}


def verify_rebuild(stage, k, m, S, s_idx, surv, l_idx, out, threads):
    """Every rebuilt byte of a device batch against the CPU oracle's rebuild
    (per-block Gauss-Jordan decode rows + the vectorised MAC) of the same
    survivor bytes and erasure patterns."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    n, e = l_idx.shape
    step = stage.rows_per_chunk((k + e) * S)
    ok = True
    for r0 in range(0, n, step):
        r1 = min(n, r0 + step)
        hs = stage.fetch("in", surv, r0, r1)
        ho = stage.fetch("out", out, r0, r1)
        want = stage.scratch("want", r1 - r0, e * S)
        O.rebuild_simd(k, m, S, s_idx[r0:r1], hs, l_idx[r0:r1], threads=threads, out=want)
        ok = ok and same_bytes(want, ho)
    return {"blocks": n, "erasures": e, "bytes_compared": n * e * S, "bit_exact": ok,
            "seconds": round(time.perf_counter() - t0, 2)}


def probe_rate(torch, codec, stream, kin, r, inp, out, launches=10, warmup=5):
    """What the memory system allows for the MAC's own traffic on this GPU
    (memo_ec_stream_probe: the same tiles and 16-byte non-temporal loads /
    stores, XOR in place of the GF arithmetic, over the same buffers; HIP
    events on `stream`).  `GBs` / `frac` (the achievable denominator): the
    read-only and the write-only launches' times added -- this mix of read
    and write streams without the cost of interleaving them.  `copy`: both
    in one launch, as a naive streaming kernel interleaves them."""
    n, S = inp.shape[0], inp.shape[1] // kin
    alg = (kin + r) * S * n
    ms = {}
    for mode in ("read", "write", "copy"):
        _, (pms,), _ = timed_steps(torch, [lambda: codec.stream_probe(kin, r, inp, out, mode)], launches,
                                   warmup, 0, None, stream)
        ms[mode] = float(np.mean(pms))
    t = ms["read"] + ms["write"]
    gbs = lambda b, x: round(b / (x * 1e-3) / 1e9, 1)  # noqa: E731
    return {"kernel": "stream_probe_kernel (the MAC's loads / stores, XOR only): read-only + write-only "
                      "launches", "GBs": gbs(alg, t), "frac": round(alg / (t * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "kernel_ms_avg": round(t, 4),
            "read": {"ms": round(ms["read"], 4), "GBs": gbs(kin * S * n, ms["read"])},
            "write": {"ms": round(ms["write"], 4), "GBs": gbs(r * S * n, ms["write"])},
            "copy": {"ms": round(ms["copy"], 4), "GBs": gbs(alg, ms["copy"]),
                     "frac": round(alg / (ms["copy"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}}


def _rate(fn, nbytes, seconds):
    """GiB/s of repeated fn() passes over ~`seconds` (at least one pass)."""
    passes, t = 0, time.perf_counter()
    while True:
        fn()
        passes += 1
        el = time.perf_counter() - t
        if el >= seconds:
            return passes * nbytes / el / 2**30, passes, el


def host_cores():
    """CPUs in this process's affinity set (the whole machine on the GPU box)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cgroup_cpus():
    """The cgroup CPU quota of this process (None: no quota)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            return max(1, q // per) if q > 0 else None
        except (OSError, ValueError):
            return None


def _omp_threads():
    try:
        return max(0, int(os.environ.get("OMP_NUM_THREADS", "0")))
    except ValueError:
        return 0


def cpu_share():
    """CPUs this process may actually keep busy: the affinity set, capped by
    the cgroup CPU quota and by OMP_NUM_THREADS when set (the GPU box gives a
    one-GPU job 16 CPUs of a 256-CPU machine; `nproc` reports 16 there)."""
    n = host_cores()
    q = _cgroup_cpus()
    if q:
        n = min(n, q)
    omp = _omp_threads()
    if omp > 0:
        n = min(n, omp)
    return n


def job_cpu_share(world):
    """CPUs of the whole job at `world` ranks on this node: the affinity set
    capped by the cgroup quota (shared by the ranks), and by
    OMP_NUM_THREADS x world where the environment gives each rank a share.
    torch.distributed.run sets OMP_NUM_THREADS=1 for ranks whose environment
    does not name one; that default is not a share and is ignored."""
    if world <= 1:
        return cpu_share()
    n = host_cores()
    q = _cgroup_cpus()
    if q:
        n = min(n, q)
    omp = _omp_threads()
    if omp > 1:
        n = min(n, omp * world)
    return max(1, n)


def cpu_threads(world=1):
    """Threads of the CPU baseline: the job's CPU share (one GPU: the
    process's share, 16 on the GPU box; N GPUs: the node share of all N
    ranks, since the baseline is the node's CPU path beside N GPUs)."""
    return max(1, job_cpu_share(world))


def cpu_baseline(k, m, B, S, seconds, gpu_parity_sample, world=1):
    """Time the CPU codecs of oracle/ on this host, on a bounded sample of
    the same workload, and cross-check them against the GPU parity of the
    same blocks.  `value` is the vectorised encode (oracle/rs_simd.c:
    GFNI+AVX-512 affine or AVX2 split-nibble, ISA-L's published x86
    techniques), the strongest CPU codec here, on the job's CPU share
    (job_cpu_share: the process's share at N = 1, the node share of all N
    ranks at N > 1; the sample grows with the threads so each has blocks),
    one core beside it, and the scalar table oracle too.  Test
    infrastructure, never the product."""
    from oracle import oracle as O
    O.build()
    threads = cpu_threads(world)
    nb = max(128, 2 * threads)
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
    nsc = min(nb, max(32, threads))
    sc_all, _, _ = _rate(lambda: O.encode(k, m, S, data[:nsc], threads=threads), nsc * B, 2.0)
    sc_one, _, _ = _rate(lambda: O.encode(k, m, S, data[:2], threads=1), 2 * B, 1.0)
    # the rebuild configs (C3): the same blocks, 4 random erasures each,
    # per-block decode rows + the vectorised MAC (oracle/rs_simd.c)
    e = min(4, m)
    s_idx, l_idx = O.erasures(SEED, 0, nb, k, m, e)
    surv = O.gather(k, m, S, data, par, s_idx)
    want = O.gather(k, m, S, data, par, l_idx)
    rout = O.aligned_empty((nb, e * S))
    O.rebuild_simd(k, m, S, s_idx, surv, l_idx, threads=threads, isa=isa, out=rout)
    ok_reb = bool(np.array_equal(rout, want))
    rv, _, _ = _rate(lambda: O.rebuild_simd(k, m, S, s_idx, surv, l_idx, threads=threads, isa=isa,
                                            out=rout), nb * B, 3.0)
    rone, _, _ = _rate(lambda: O.rebuild_simd(k, m, S, s_idx[:16], surv[:16], l_idx[:16], threads=1,
                                              isa=isa, out=rout[:16]), 16 * B, 1.0)
    return {"value": round(v, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "RS(%d,%d) encode, %d x %d-byte blocks x %d passes (%.1f s), vectorised C port "
                      "(%s, streaming stores) on %d threads (the job's CPU share at %d GPU%s; %d "
                      "CPUs in the affinity set); 1-core %.3f GiB/s; scalar table oracle %.3f GiB/s "
                      "on %d threads, %.3f on 1; bit-exact vs GPU on %d blocks: %s"
                      % (k, m, nb, B, passes, el, O.SIMD_ISA[isa], threads, world,
                         "" if world == 1 else "s", host_cores(), one, sc_all, threads, sc_one, nchk,
                         ok_simd and ok_scalar),
            "isa": O.SIMD_ISA[isa], "single_core": round(one, 3), "n_gpus": world,
            "per_gpu_share": round(threads / world, 2),
            "cpu_share": cpu_share(), "affinity_cpus": host_cores(),
            "rebuild": {"value": round(rv, 3), "single_core": round(rone, 3), "threads": threads,
                        "erasures": e, "bit_exact": ok_reb,
                        "sample": "RS(%d,%d) rebuild of the same %d blocks, %d random erasures each "
                                  "(decode rows by Gauss-Jordan, memoised per pattern, + vectorised MAC)"
                                  % (k, m, nb, e)},
            "scalar_oracle": {"value": round(sc_all, 3), "single_core": round(sc_one, 3)},
            "bit_exact_vs_gpu": ok_simd and ok_scalar}


def c1_case(torch, ec, codec, stream, world=1):
    """BASELINE.json configs[0] (C1): RS(3,2) encode + rebuild (e = 1 and 2
    random erasures per block) of 1000 x 64 KiB blocks.  The CPU oracle
    (scalar, 16 host threads; the reference-runnable case) and the
    vectorised port (the cpu_baseline's kind, same threads) are timed beside
    the GPU on the same bytes, and every rebuilt shard is compared across
    the three (whole batch, bit-exact)."""
    from oracle import oracle as O
    k, m, B, n = 3, 2, 65536, 1000
    S = ec.shard_size(B, k)
    threads = cpu_threads(world)
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    t0 = time.perf_counter()
    par = O.encode(k, m, S, data, threads=threads)
    cpu_enc = time.perf_counter() - t0
    d = torch.from_numpy(data).cuda()
    p = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    _, (ek,), _ = timed_steps(torch, [lambda: codec.encode(k, m, d, p)], 20, 20, 0, None, stream)
    ok = bool(np.array_equal(p.cpu().numpy(), par))
    # the vectorised port (GFNI/AVX-512 or AVX2, the cpu_baseline's kind) on
    # the same threads and bytes beside the scalar oracle: the fair CPU time
    simd_par, isa = O.encode_simd(k, m, S, data, threads=threads)
    t0 = time.perf_counter()
    O.encode_simd(k, m, S, data, threads=threads, isa=isa, out=simd_par)
    simd_enc = time.perf_counter() - t0
    ok = ok and bool(np.array_equal(simd_par, par))
    out = {"workload": "RS(3,2) encode + rebuild (e=1, e=2), 1000 x 65536-byte blocks (BASELINE.json C1)",
           "cpu_threads": threads, "cpu_kind": "port (scalar table oracle)",
           "cpu_simd_kind": "port (%s)" % O.SIMD_ISA.get(isa, str(isa)),
           "encode": {"cpu_ms": round(cpu_enc * 1e3, 3), "cpu_simd_ms": round(simd_enc * 1e3, 3),
                      "gpu_ms": round(float(np.median(ek)), 4)}}
    for e in (1, 2):
        s_idx, l_idx = O.erasures(SEED, 0, n, k, m, e)
        surv = O.gather(k, m, S, data, par, s_idx)
        t0 = time.perf_counter()
        want = O.rebuild(k, m, S, s_idx, surv, l_idx, threads=threads)
        cpu_reb = time.perf_counter() - t0
        simd_out, _ = O.rebuild_simd(k, m, S, s_idx, surv, l_idx, threads=threads, isa=isa)
        t0 = time.perf_counter()
        O.rebuild_simd(k, m, S, s_idx, surv, l_idx, threads=threads, isa=isa, out=simd_out)
        simd_reb = time.perf_counter() - t0
        ok = ok and bool(np.array_equal(simd_out, want))
        sd, ld, sv = (torch.from_numpy(x).cuda() for x in (s_idx, l_idx, surv))
        o = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        _, (rk,), _ = timed_steps(torch, [lambda: codec.rebuild(k, m, sd, sv, ld, o)], 20, 20, 0,
                                  None, stream)
        codec.synchronize()
        ok = ok and bool(np.array_equal(o.cpu().numpy(), want))
        out["rebuild_e%d" % e] = {"cpu_ms": round(cpu_reb * 1e3, 3), "cpu_simd_ms": round(simd_reb * 1e3, 3),
                                  "gpu_ms": round(float(np.median(rk)), 4)}
    out["bit_exact"] = ok
    return out


def end_to_end(torch, ec, codec, data, par, k, m, B, n):
    """PCIe-inclusive rates (blocks start and end in host memory: RPC socket
    in, silos/peers out); 3-stage pipeline, 64 MiB batches.  Never `value`."""
    S = ec.shard_size(B, k)
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
    res = {"workload": "RS(%d,%d) encode, %d x %d-byte blocks from host memory, parity back to "
                       "host memory (HtoD + kernel + DtoH, 3-stage stream pipeline)" % (k, m, ne, B),
           "unit": "GiB/s", "pinned": e2e["pinned"], "pageable": e2e["pageable"]}
    # One-block host calls, as the plugin issues them for a lone store or a
    # degraded read (pageable elle::Buffer in, out): latency, not rate.
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
    lat["note"] = ("median of 200 one-block calls from pageable host memory (copy in, kernels, "
                   "copy out, synchronous), RS(%d,%d)" % (k, m))
    return res, lat


def sha_digests_ok(msgs, digs, idx, bb, threads):
    """Digests digs[i] == SHA-256(64 zero bytes || msgs[i, :bb]) for the rows
    idx (host arrays), by hashlib on a thread pool (it releases the GIL on
    large inputs)."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    pre = bytes(64)

    def one(i):
        return hashlib.sha256(pre + msgs[i, :bb].tobytes()).digest() == digs[i].tobytes()
    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        return all(ex.map(one, idx))


def sha_lines(torch, codec, stream, data, n, B, threads=1):
    """sha256_kernel (CHB::_hash_address, CHB.cc:264-289), one lane per block:
    the C2 batch (4096 x 1 MiB, every digest checked with hashlib) and
    1,048,576 x 4 KiB blocks (every 64th digest checked).  Not a roofline
    line: 4096 lanes cannot fill the chip, and the hash is issue-bound."""
    import hashlib
    res = {}
    for name, nb, bb, every in [("C2 batch, 1 MiB blocks", n, B, 1), ("4 KiB blocks", 1 << 20, 4096, 64)]:
        msg = data if bb == B else torch.empty((nb, bb), dtype=torch.uint8, device="cuda")
        stride = msg.shape[1]
        if bb != B:
            codec.fill_blocks(SEED, 0, nb, bb, 1, bb, msg)
        pre = torch.zeros((nb, 64), dtype=torch.uint8, device="cuda")  # salt || owner
        dig = torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
        fn = lambda: codec.sha256(msg, dig, prefix=pre, uniform_len=bb, msg_stride=stride)  # noqa
        _, (kms,), _ = timed_steps(torch, [fn], 5, 1, 0, None, stream)
        ms = float(np.mean(kms))
        idx = np.arange(0, nb, every)
        ok = sha_digests_ok(msg[idx].cpu().numpy(), dig[idx].cpu().numpy(), range(len(idx)), bb, threads)
        one = msg[0, :bb].cpu().numpy().tobytes()
        t = time.perf_counter()
        reps = max(1, (64 << 20) // bb)
        for _ in range(reps):
            hashlib.sha256(one).digest()
        cpu = reps * bb / (time.perf_counter() - t) / 1e9
        res[name] = {"blocks": nb, "block_bytes": bb, "kernel_ms": round(ms, 3),
                     "GBs": round(nb * (bb + 64) / (ms * 1e-3) / 1e9, 1), "bit_exact": ok,
                     "checked": int(len(idx)), "cpu_1core_GBs": round(cpu, 2)}
        del pre, dig
        if bb != B:
            del msg
    return {"workload": "batched SHA-256(salt||owner||data) = CHB addresses (CHB.cc:264-289), "
                        "one lane per block", **res}


def _visible_device(local):
    """The device string a child process must see to use this rank's GPU."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            ids = [x for x in v.split(",") if x.strip()]
            return var, ids[local] if local < len(ids) else ids[0]
    return "HIP_VISIBLE_DEVICES", str(local)


def pmc_traffic(args, result, local, world):
    """roofline.traffic measured by this run: two rocprofv3 counter passes
    (FETCH_SIZE, then WRITE_SIZE -- they cannot share a pass on gfx950) over
    a short run of the same step on this rank's GPU, each a child process
    started after the timed region.  HBM bytes per launch = 2 * FETCH_SIZE +
    WRITE_SIZE (KiB units): on gfx950 FETCH_SIZE reports half the bytes of a
    wide coalesced streaming read, WRITE_SIZE is exact for 16-byte-per-lane
    stores (MI355X_MICROARCH.md, HBM).  The rebuild's traffic is its
    kernels' per step (decode rows + MAC, or the fused kernel)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    k, m, B, n, e = args.k, args.m, args.block_bytes, args.blocks, args.erasures
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    env = {x: v for x, v in os.environ.items()
           if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "MASTER_ADDR", "MASTER_PORT") and not x.startswith("TORCHELASTIC")}
    if world > 1 and not args.same_device:
        var, dev = _visible_device(local)
        env[var] = dev
    child = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", "3", "--warmup", "1",
             "--settle-ms", "0", "--no-small", "--no-cpu", "--no-e2e", "--no-pmc", "--no-verify",
             "--no-c5", "--no-plugin", "--no-sha",
             "--k", str(k), "--m", str(m), "--block-bytes", str(B), "--blocks", str(n),
             "--erasures", str(e)]

    def kind(name):
        if "gf_mac_images_kernel" in name:  # the rebuild MAC over per-block table images
            return "rebuild"
        if "gf_mac_kernel" in name:
            return "rebuild" if name.split("(")[0].rstrip(">").rstrip().endswith("true") else "encode"
        if "gf_rebuild_kernel" in name or "decode_" in name:
            return "rebuild_" + ("fused" if "gf_rebuild_kernel" in name else "decode")
        return None

    tmp = tempfile.mkdtemp(prefix="memo_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    per = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            r = subprocess.run([rocprof, "--pmc", counter, "-d", d, "-o", "pmc", "-f", "csv", "--"] + child,
                               env=env, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                               timeout=150)
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                raise RuntimeError("rocprofv3 --pmc %s: rc %d, %s" % (counter, r.returncode,
                                                                      r.stderr.decode(errors="replace")[-300:]))
            vals = {}
            for f in files:
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        kd = kind(row.get("Kernel_Name", ""))
                        if kd:
                            vals.setdefault(kd, []).append(float(row["Counter_Value"]))
            if not vals.get("encode"):
                raise RuntimeError("no encode kernel in the %s counter files" % counter)
            per[counter] = vals
    except (OSError, RuntimeError, subprocess.SubprocessError, KeyError, ValueError) as ex:
        for key in ("roofline", "roofline_rebuild"):
            if key in result:
                result[key]["traffic"] = None
                result[key]["traffic_note"] = "counter passes failed: %s" % str(ex)[:300]
        return
    finally:
        shutil.rmtree(tmp, ignore_errors=True)

    def kb(counter, kd):
        v = per.get(counter, {}).get(kd, [])
        return float(np.median(v)) if v else 0.0

    def traffic(kinds):
        return int(round(sum(2 * kb("FETCH_SIZE", kd) + kb("WRITE_SIZE", kd) for kd in kinds) * 1024))

    src = ("measured by this run: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (separate "
           "child runs of the same step, 3 steps each, median launch), bytes = (2*FETCH_SIZE + "
           "WRITE_SIZE) * 1024; build %s" % result["build_id"][:16])
    enc = traffic(["encode"])
    result["roofline"]["traffic"] = enc
    result["roofline"]["traffic_ratio"] = round(enc / result["roofline"]["bytes_per_launch"], 4)
    result["roofline"]["traffic_source"] = src
    if "roofline_rebuild" in result:
        kinds = [x for x in ("rebuild_decode", "rebuild", "rebuild_fused") if per["FETCH_SIZE"].get(x)]
        rb = traffic(kinds)
        result["roofline_rebuild"]["traffic"] = rb
        result["roofline_rebuild"]["traffic_ratio"] = round(rb / result["roofline_rebuild"]["bytes_per_launch"], 4)
        result["roofline_rebuild"]["traffic_kernels"] = kinds
        result["roofline_rebuild"]["traffic_source"] = src


PLUGIN_BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host", "_build", "bench_plugin")
# (blocks, block bytes): the 4 KiB-block point of SURVEY.md 8(d) and 1 MiB
# blocks, through the whole consensus (place, silo writes, multi-fetch,
# eviction + repair) beside replication; a few seconds each.
PLUGIN_SIZES = [(16384, 4096), (512, 1 << 20)]
PLUGIN_KEYS = ("store_GiBs", "fetch_GiBs", "degraded_fetch_GiBs", "repair_GiBs")
PLUGIN_REPS = 5


def spread(samples):
    """{median, min, max, n, samples} of one rate's repetitions."""
    v = sorted(float(x) for x in samples)
    n = len(v)
    med = v[n // 2] if n % 2 else (v[n // 2 - 1] + v[n // 2]) / 2
    return {"median": round(med, 3), "min": round(v[0], 3), "max": round(v[-1], 3), "n": n,
            "samples": [round(float(x), 3) for x in samples]}


def plugin_aggregate(d):
    """The child's per-repetition lists -> {median, min, max, n} per rate, and
    the erasure / replication ratio of each repetition (the sides ran back
    to back in that repetition, so the ratio cancels box drift) for store
    and fetch: against replication through validating peers (`ratio`) and
    through plain peers (`ratio_unvalidated`, the rounds 1-5 baseline)."""
    er, rp = dict(d.get("erasure", {})), dict(d.get("replication", {}))
    ru = dict(d.get("replication_unvalidated", {}))
    for side in (er, rp, ru):
        for key, val in list(side.items()):
            if key.endswith("_GiBs") and isinstance(val, list) and val:
                side[key] = spread(val)

    def ratios(other):
        out = {}
        for key in ("store_GiBs", "fetch_GiBs"):
            a, b = er.get(key), other.get(key)
            if isinstance(a, dict) and isinstance(b, dict) and a["n"] == b["n"]:
                per = [x / y for x, y in zip(a["samples"], b["samples"]) if y > 0]
                if len(per) == a["n"]:
                    out[key.replace("_GiBs", "")] = spread(per)
        return out
    return er, rp, ru, ratios(rp), ratios(ru)


def plugin_lines(binary=PLUGIN_BIN, sizes=PLUGIN_SIZES, timeout=240, reps=PLUGIN_REPS):
    """The plugin level (host/erasure_consensus.cc, the drop-in for the
    reference's Consensus, src/memo/model/doughnut/Consensus.hh:24-174): child runs
    of host/tests/bench_plugin.cc, each on in-process memory-silo nodes, which
    exit non-zero unless every healthy, degraded and post-repair fetch returns
    bytes whose SHA-256 matches the block's CHB address and nothing is left
    unrecoverable.  Each child runs erasure and replication interleaved `reps`
    times on fresh nodes; a row carries {median, min, max, n} per rate and
    the per-repetition erasure / replication ratios (`ratio`).  Host-bound
    (the place step and silo copies), not a kernel roofline line; it runs
    after the timed region."""
    import subprocess
    out = {}
    for nb, bb in sizes:
        key = "%dx%d" % (nb, bb)
        try:
            r = subprocess.run([binary, str(nb), str(bb), str(reps)], stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, timeout=timeout)
            line = r.stdout.decode(errors="replace").strip().splitlines()
            d = json.loads(line[-1]) if line else {}
            er, rp, ru, ratio, ratio_u = plugin_aggregate(d)
            row = {"ok": r.returncode == 0 and all(x in er for x in PLUGIN_KEYS),
                   "reps": d.get("reps"), "erasure": er, "replication": rp, "ratio": ratio}
            if ru:
                row["replication_unvalidated"] = ru
                row["ratio_unvalidated"] = ratio_u
            if not row["ok"]:
                row["note"] = "rc %d: %s" % (r.returncode, r.stderr.decode(errors="replace")[-300:])
        except (OSError, subprocess.SubprocessError, ValueError, IndexError) as ex:
            row = {"ok": False, "note": str(ex)[:300]}
        out[key] = row
    return out


SMALL_PMC = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_ACTIVE_INST_ANY",
             "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]


def pmc_small(args, result, local, world):
    """One rocprofv3 counter pass over a child run of the 4 KiB lines (the
    per-block-pattern rebuild and the encode of the same blocks, both codes)
    and, per kernel, what bounds it: valu_busy = SQ_INSTS_VALU x 2 cycles (a
    wave64 VALU instruction holds a SIMD-32 for 2) over the 1024 SIMDs'
    cycles (GRBM_GUI_ACTIVE / 8 XCDs = the dispatch's cycles at its own
    clock, MI355X_MICROARCH.md), and each wave's split into issuing,
    issue-stalled and parked (waitcnt / barrier) cycles."""
    import csv
    import glob
    import re
    import shutil
    import subprocess
    import tempfile
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    env = {x: v for x, v in os.environ.items()
           if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "MASTER_ADDR", "MASTER_PORT") and not x.startswith("TORCHELASTIC")}
    if world > 1 and not args.same_device:
        var, dev = _visible_device(local)
        env[var] = dev
    # clocks settled first (150 ms of untimed steps), as the timed lines are
    child = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--small-only", "--steps", "4",
             "--warmup", "2", "--settle-ms", "150"]
    tmp = tempfile.mkdtemp(prefix="memo_pmc_small_", dir=os.environ.get("TMPDIR", "/tmp"))
    vals = {}
    try:
        d = os.path.join(tmp, "sq")
        r = subprocess.run([rocprof, "--pmc"] + SMALL_PMC + ["-d", d, "-o", "pmc", "-f", "csv", "--"] + child,
                           env=env, cwd=tmp, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=240)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            raise RuntimeError("rocprofv3: rc %d, %s" % (r.returncode, r.stderr.decode(errors="replace")[-300:]))
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    mm = re.search(r"gf_mac_kernel<(\d+), (\d+), \w+, (true|false)>", name)
                    md = re.search(r"decode_\w*kernel<(\d+)", name)
                    if mm:
                        key = (int(mm.group(1)), "rebuild MAC" if mm.group(3) == "true" else "encode MAC")
                    elif md:
                        key = (int(md.group(1)), "decode rows")
                    else:
                        continue
                    dd = vals.setdefault(key, {}).setdefault((row.get("Dispatch_Id"), ), {})
                    dd[row["Counter_Name"]] = float(row["Counter_Value"])
                    try:
                        dd["_ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                    except (KeyError, ValueError):
                        pass
        if not vals:
            raise RuntimeError("no codec kernel in the counter files")
    except (OSError, RuntimeError, subprocess.SubprocessError, KeyError, ValueError) as ex:
        result.setdefault("rebuild_small", {})["counters_note"] = "counter pass failed: %s" % str(ex)[:300]
        return
    finally:
        shutil.rmtree(tmp, ignore_errors=True)

    def summary(disp):
        def med(c):
            v = [x[c] for x in disp.values() if c in x]
            return float(np.median(v)) if v else 0.0
        waves = med("SQ_WAVES") or 1.0
        cycles = med("GRBM_GUI_ACTIVE") / 8
        ns = med("_ns")
        out = {"valu_busy": round(med("SQ_INSTS_VALU") * 2 / (1024 * cycles), 4) if cycles else None,
               "clock_GHz": round(cycles / ns, 3) if ns else None,
               "cycles_per_wave": round(4 * med("SQ_WAVE_CYCLES") / waves),
               "valu_per_wave": round(med("SQ_INSTS_VALU") / waves, 1),
               "salu_per_wave": round(med("SQ_INSTS_SALU") / waves, 1),
               "lds_per_wave": round(med("SQ_INSTS_LDS") / waves, 1),
               "issuing_cycles_per_wave": round(4 * med("SQ_ACTIVE_INST_ANY") / waves),
               "issue_stalled_cycles_per_wave": round(4 * med("SQ_WAIT_INST_ANY") / waves),
               "parked_cycles_per_wave": round(4 * med("SQ_WAIT_ANY") / waves),
               "dispatches": len(disp)}
        return out

    for (kc, kind), disp in sorted(vals.items()):
        name = {16: "RS(16,4)", 10: "RS(10,4)"}.get(kc)
        if name and name in result.get("rebuild_small", {}):
            result["rebuild_small"][name].setdefault("counters", {})[kind] = summary(disp)
    result.setdefault("rebuild_small", {})["counters_source"] = (
        "rocprofv3 --pmc %s, one pass over a child run of the same 4 KiB lines (4 steps after 150 ms of "
        "untimed ones), per-dispatch "
        "medians; valu_busy = SQ_INSTS_VALU * 2 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8); clock_GHz = "
        "GRBM_GUI_ACTIVE / 8 / the dispatch's duration (counter passes serialise dispatches and run "
        "a few %% below the unprofiled clock); *_cycles_per_wave from the quad-cycle SQ counters" %
        " ".join(SMALL_PMC))


def merge_extras(result, extras):
    """Fold the ranks' side measurements (one dict per rank, rank order) into
    the contract line (pure: tested on CPU): the achievable rate of the
    encode's traffic on each rank's GPU (memo_ec_stream_probe), the
    whole-batch oracle comparisons of every rank, and the PCIe end-to-end
    rates."""
    world = len(extras)
    x0 = extras[0]
    roof = result["roofline"]
    if "probe" in x0:
        pr = x0["probe"]
        roof["achievable"] = pr
        roof["frac_of_achievable"] = round(roof["achieved"] / pr["GBs"], 4)
        if "roofline_rebuild" in result:
            rr = result["roofline_rebuild"]
            rr["achievable_GBs"] = pr["GBs"]
            rr["frac_of_achievable"] = round(rr["achieved"] / pr["GBs"], 4)
        if world > 1:
            roof["achievable_per_rank_GBs"] = [x["probe"]["GBs"] for x in extras]
    if "oracle" in x0:
        par = {}
        for key in x0["oracle"]:
            checks = [x["oracle"][key] for x in extras]
            par[key] = dict(checks[0])
            par[key]["bit_exact"] = all(c["bit_exact"] for c in checks)
            par[key]["blocks"] = sum(c["blocks"] for c in checks)
            par[key]["bytes_compared"] = sum(c["bytes_compared"] for c in checks)
            par[key]["seconds"] = max(c["seconds"] for c in checks)
            if world > 1:
                par[key]["ranks"] = len(checks)
        result["oracle_parity"] = par
    if "e2e" not in x0:
        return result
    result["end_to_end"] = dict(x0["e2e"])
    result["host_call_latency"] = x0["lat"]
    if world > 1:
        result["end_to_end"]["per_rank"] = [
            {"rank": i, "pinned": x["e2e"]["pinned"]["value"], "pageable": x["e2e"]["pageable"]["value"]}
            for i, x in enumerate(extras)]
        result["end_to_end"]["node_sum"] = {
            kind: round(sum(x["e2e"][kind]["value"] for x in extras), 3) for kind in ("pinned", "pageable")}
        result["end_to_end"]["note"] = ("every rank streams over its own GPU's PCIe link at the same "
                                        "time; node_sum adds the ranks' rates")
    return result


def check_devices(rows, same_device):
    """Every rank ran on its own GPU: the ranks' PCI bus ids and UUIDs
    (memo_ec_device_identity) are pairwise distinct, unless the run asked
    for one shared device (--same-device rehearsals).  Raises otherwise: a
    node figure from ranks sharing a GPU is not a scaling result."""
    ids = [r.get("device_identity") for r in rows]
    if same_device or len(rows) < 2:
        return
    if any(i is None for i in ids):
        raise RuntimeError("bench: a rank reported no device identity")
    for key in ("pci_bus_id", "uuid"):
        seen = {}
        for r, i in zip(rows, ids):
            if i[key] in seen:
                raise RuntimeError("bench: ranks %d and %d ran on the same GPU (%s %s)"
                                   % (seen[i[key]], r["rank"], key, i[key]))
            seen[i[key]] = r["rank"]


# Legs of the default line that run at N = 1 only (single-GPU workloads, or
# host-side lines that do not depend on N): named in the N > 1 line itself.
N1_ONLY_LEGS = [("rebuild_small", "no_small", "1,048,576 x 4 KiB rebuilds: a single-GPU workload"),
                ("c5_mixed", "no_c5", "BASELINE.json C5 is quoted on 1 GPU"),
                ("plugin", "no_plugin", "host-side plugin lines, independent of N"),
                ("sha256", "no_sha", "single-GPU SHA-256 lines"),
                ("sweep", None, "BASELINE.json C5 sweep is quoted on 1 GPU (--sweep)")]


def skipped_at_n(args, world):
    """{leg: reason} of the legs an N > 1 line leaves out (empty at N = 1);
    legs the run's flags turned off are not listed."""
    if world <= 1:
        return {}
    out = {}
    for leg, flag, why in N1_ONLY_LEGS:
        if flag is None:
            if getattr(args, "sweep", False):
                out[leg] = why
        elif not getattr(args, flag):
            out[leg] = why
    return out


# Rates behind post_timed_seconds, measured on the GPU boxes: the oracle
# port's single-core encode (BENCH_r05.json cpu_baseline.single_core: 27.1
# GiB/s; its rebuild is faster), the pinned device-to-host rate one link
# gives a staged 256 MiB chunk while every link of the node is busy (DESIGN
# §6: 49.4 GiB/s both directions on one link; half of it taken here), the
# seconds of one rocprofv3 counter pass (a child bench.py: torch import,
# fill, a few launches; tens of seconds on a fresh box), the PCIe
# end-to-end leg and the in-library stream probe.
POST_RATES = {"oracle_core_GiBs": 27.0, "dtoh_GiBs": 20.0, "pmc_pass_s": 60.0, "e2e_s": 10.0,
              "probe_s": 3.0, "c1_s": 5.0, "startup_s": 120.0}


def post_timed_seconds(args, world, threads_per_rank, S, rates=POST_RATES):
    """Estimated seconds a rank spends outside the timed steps at `world`
    ranks with `threads_per_rank` CPU threads each (main: the job's CPU share
    split over the ranks): start-up (torch import, inputs), the stream probe,
    the whole-batch oracle checks of its own C2 / C3 batches (staged over its
    own link, recomputed on its threads), the PCIe end-to-end leg, and on
    rank 0 the CPU baseline, C1 and the counter passes.  The N = 1-only legs
    (4 KiB lines, C5, plugin, SHA-256) are not run at N > 1.  Returns
    {"rank": s, "rank0": s, "legs": {...}} to hold against --rank-timeout."""
    k, m, n, e = args.k, args.m, args.blocks, args.erasures
    gib = float(1 << 30)
    legs = {"startup": rates["startup_s"], "probe": rates["probe_s"]}
    if not args.no_verify:
        core = rates["oracle_core_GiBs"] * max(1, threads_per_rank)
        c2 = n * (k + m) * S / gib / rates["dtoh_GiBs"] + n * k * S / gib / core
        c3 = n * (k + e) * S / gib / rates["dtoh_GiBs"] + n * k * S / gib / core if e > 0 else 0.0
        legs["oracle_checks"] = c2 + c3
    if not args.no_e2e:
        legs["end_to_end"] = rates["e2e_s"]
    rank = sum(legs.values())
    r0 = dict(legs)
    if not args.no_cpu:
        r0["cpu_baseline"] = args.cpu_seconds * 1.5  # the timed sample, its setup and the scalar oracle
        r0["c1"] = rates["c1_s"]
    if not args.no_pmc:
        r0["counter_passes"] = 2 * rates["pmc_pass_s"]
    if world == 1:
        if not args.no_small:
            r0["rebuild_small"] = 60.0
        if not args.no_c5:
            r0["c5_mixed"] = 30.0
        if not args.no_plugin:
            r0["plugin"] = 120.0
        if not args.no_sha:
            r0["sha256"] = 20.0
    return {"rank": round(rank, 2), "rank0": round(sum(r0.values()), 2),
            "legs": {k_: round(v, 2) for k_, v in r0.items()}}


def assemble(args, world, rows, wall_max, S):
    """The contract line from the ranks' rows (pure: tested on CPU)."""
    from memo_amd.partition import node_report
    check_devices(rows, args.same_device)
    k, m, B, n, e, K = args.k, args.m, args.block_bytes, args.blocks, args.erasures, args.steps
    r0 = rows[0]
    step_payload = n * B * (2 if e > 0 else 1)
    value = world * step_payload * K / wall_max / 2**30
    enc_alg = (k + m) * S * n
    enc = r0["encode"]
    roof = {"bound": "hbm", "kernel": "gf_mac_kernel (encode)", "achieved": enc["achieved"],
            "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": enc["frac"], "traffic": None,
            "bytes_per_launch": enc_alg,
            "read_only_frac": round(k * S * n / (enc["kernel_ms_avg"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            **{x: enc[x] for x in ("kernel_ms_avg", "kernel_ms_min", "kernel_ms_median",
                                   "kernel_ms_first_last")},
            "kernel_ms_max_over_ranks": round(max(r["encode"]["kernel_ms_avg"] for r in rows), 4)}
    res = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(wall_max / K * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "RS(%d,%d) encode (BASELINE.json C2) + rebuild with %d random erasures "
                               "per block (C3) of %d x %d-byte blocks per GPU%s; step = one encode "
                               "launch + one rebuild launch" % (k, m, e, n, B,
                                                                "" if world == 1 else " (C4 at N=8)"),
                   "k": k, "m": m, "block_bytes": B, "blocks_per_gpu": n, "shard_bytes": S,
                   "erasures": e, "global_blocks": n * world,
                   "parallelism": "block-index partition x%d, no collective on data" % world},
        "roofline": roof,
        "warmup_steps_run": r0["warmup_steps_run"],
        "encode": {"value": round(world * n * B * K / wall_max / 2**30, 3) if e <= 0 else None,
                   "GiBs_kernel": round(n * B / (enc["kernel_ms_avg"] * 1e-3) / 2**30, 1), **enc},
    }
    if e > 0:
        reb = r0["rebuild"]
        rb_alg = (k + e) * S * n
        res["encode"].pop("value")
        res["rebuild"] = {"GiBs_kernel": round(n * B / (reb["kernel_ms_avg"] * 1e-3) / 2**30, 1),
                          "bytes_per_launch": rb_alg, "round_trip_bit_exact": all(
                              r["rebuild_bit_exact"] for r in rows), **reb}
        res["roofline_rebuild"] = {"bound": "hbm", "kernel": r0["rebuild_kernel"],
                                   "achieved": reb["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                   "frac": reb["frac"], "traffic": None, "bytes_per_launch": rb_alg,
                                   "kernel_ms_avg": reb["kernel_ms_avg"]}
    per = [{"rank": r["rank"], "device": r["device"], "payload_bytes": r["payload_bytes"],
            "seconds": r["device_seconds"]} for r in rows]
    rep = node_report(per)
    res["ranks"] = {"per_gpu": [{"rank": r["rank"], "device": r["device"],
                                 **r.get("device_identity", {}),
                                 "GiBs": rep["per_gpu_GiBs"][i],
                                 "encode_kernel_ms": r["encode"]["kernel_ms_avg"],
                                 "encode_frac": r["encode"]["frac"],
                                 **({"rebuild_kernel_ms": r["rebuild"]["kernel_ms_avg"],
                                     "rebuild_frac": r["rebuild"]["frac"]} if e > 0 else {})}
                                for i, r in enumerate(rows)],
                    "node_sum_GiBs": rep["node_sum_GiBs"],
                    "distinct_devices": len({(r.get("device_identity") or {}).get("uuid", r["device"])
                                             for r in rows}),
                    "note": "per-GPU GiB/s = that rank's payload / its own kernel time (HIP events); "
                            "node sum = all payload / the slowest rank's kernel time; `value` = all "
                            "payload / the job's wall time between barriers; pci_bus_id / uuid: "
                            "memo_ec_device_identity of the rank's GPU (distinct ranks on distinct "
                            "GPUs unless --same-device)"}
    if world > 1:
        res["skipped_at_n"] = skipped_at_n(args, world)
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # Start the N ranks here, before anything touches a GPU (children,
        # never an exec), one per device; each rank re-enters main().
        from memo_amd.partition import launch_local_ranks
        # A rank that hangs is killed (by PID) after --rank-timeout seconds
        # and the launch exits non-zero; the others stop with it.
        sys.exit(launch_local_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus,
                                    same_device=args.same_device, timeout=args.rank_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist_mod
        # gloo on the host: the barrier and the max/gather of timings only.
        # Its connect messages ("[Gloo] Rank r is connected to ...") are
        # written to stdout; stdout carries only rank 0's JSON line, so they
        # go to stderr.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            import datetime
            # a rank that never reaches a collective fails the others after
            # --rank-timeout seconds instead of gloo's 30-minute default
            dist_mod.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.rank_timeout))
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        dist = dist_mod
    if torch.cuda.device_count() <= local:
        raise SystemExit("bench.py: rank %d needs cuda:%d, %d visible" % (rank, local,
                                                                          torch.cuda.device_count()))
    torch.cuda.set_device(local)
    from memo_amd import ec
    from memo_amd.partition import weak_range

    k, m, B, n, e = args.k, args.m, args.block_bytes, args.blocks, args.erasures
    S = ec.shard_size(B, k)
    # A dedicated (non-null) stream: the codec enqueues on it and the HIP
    # events that time each launch are recorded on the same stream.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    codec = ec.Codec(local)
    codec.set_stream(stream)
    assert codec.stream == stream.cuda_stream and stream.cuda_stream
    if args.small_only:  # the child of pmc_small: the 4 KiB lines, nothing else
        rebuild_small(torch, ec, codec, stream, args.steps, args.warmup, args.settle_ms, uniform=False)
        codec.close()
        return

    data = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    par = torch.empty((n, m * S), dtype=torch.uint8, device="cuda")
    first_block, _ = weak_range(n, rank)  # rank r owns blocks [r*n, (r+1)*n)
    codec.fill_blocks(SEED, first_block, n, B, k, S, data)
    fns = [lambda: codec.encode(k, m, data, par)]
    if e > 0:
        codec.encode(k, m, data, par)
        s_idx, l_idx = ec.erasures(SEED, first_block, n, k, m, e)
        sd = torch.from_numpy(s_idx).cuda()
        ld = torch.from_numpy(l_idx).cuda()
        surv = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, data, par, sd, surv)
        out = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        want = torch.empty((n, e * S), dtype=torch.uint8, device="cuda")
        codec.gather_shards(k, m, S, n, data, par, ld, want)
        fns.append(lambda: codec.rebuild(k, m, sd, surv, ld, out))
    torch.cuda.synchronize()

    log("rank %d: inputs resident, timing %d steps" % (rank, args.steps))
    wall, kms, done = timed_steps(torch, fns, args.steps, args.warmup, args.settle_ms, dist, stream)
    codec.synchronize()
    row = {"rank": rank, "device": local, "device_identity": ec.device_identity(local),
           "warmup_steps_run": done,
           "payload_bytes": n * B * len(fns) * args.steps,
           "device_seconds": sum(sum(x) for x in kms) * 1e-3,
           "encode": kstats(kms[0], (k + m) * S * n)}
    if e > 0:
        row["rebuild"] = kstats(kms[1], (k + e) * S * n)
        row["rebuild_bit_exact"] = bool(torch.equal(out, want))
        row["rebuild_kernel"] = codec.rebuild_kernel_name(n, k, S, e)
        del want
    rows = [row]
    wall_max = wall
    if dist is not None:
        rows = [None] * world
        dist.all_gather_object(rows, row)
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall_max = float(t.item())
    result = assemble(args, world, rows, wall_max, S)

    if args.no_pmc:
        for key in ("roofline", "roofline_rebuild"):
            if key in result:
                result[key]["traffic_note"] = "not measured (--no-pmc)"
    result["build_id"] = ec.build_id()
    result["build_matches_sources"] = result["build_id"] == ec.source_id()

    # ---- after the timed steps and their closing barrier: the baselines,
    # checks and side measurements, at every N.  Every rank measures its own
    # GPU (the achievable rate of the encode's traffic, PCIe end-to-end rate
    # over its own link) and compares its own whole batch with the CPU
    # oracle, concurrently; rank 0 alone times the CPU baseline and the
    # counter passes while the others wait at the final barrier.
    extra = {}
    # What the memory system allows for this exact traffic (SURVEY.md 8(d)'s
    # "measured" reference): the encode's tiles and loads/stores, no GF math.
    scratch = torch.empty_like(par)
    extra["probe"] = probe_rate(torch, codec, stream, k, m, data, scratch)
    del scratch
    vthreads = max(1, cpu_threads(world) // world)
    if not args.no_verify:
        # Whole-batch parity with the CPU oracle (oracle/rs_simd.c): every
        # parity byte of the timed encode (C2) and every shard the timed
        # rebuild produced (C3, this batch's path), on this rank's blocks.
        log("rank %d: whole-batch oracle comparison" % rank)
        stage = HostStage(torch)
        extra["oracle"] = {"C2_encode": verify_encode(stage, k, m, S, data, par, vthreads)}
        if e > 0:
            vr = verify_rebuild(stage, k, m, S, s_idx, surv, l_idx, out, vthreads)
            vr["path"] = codec.rebuild_path(n, k, S, e)
            extra["oracle"]["C3_rebuild"] = vr
        del stage
    if e > 0:
        del surv, out
    if not args.no_e2e:
        if dist is not None:
            dist.barrier()  # all links busy at once, as on a node serving every GPU
        extra["e2e"], extra["lat"] = end_to_end(torch, ec, codec, data, par, k, m, B, n)
        codec.set_stream(stream)
    extras = [extra]
    if dist is not None:
        extras = [None] * world
        dist.all_gather_object(extras, extra)
    merge_extras(result, extras)
    log("rank %d: timed steps done, side measurements" % rank)
    checks = [v["bit_exact"] for v in result.get("oracle_parity", {}).values()]
    if world == 1:
        stage = None if args.no_verify else HostStage(torch)
        if not args.no_small:
            result["rebuild_small"] = rebuild_small(torch, ec, codec, stream, args.steps, args.warmup,
                                                    args.settle_ms, stage, vthreads)
            for v in result["rebuild_small"].values():
                checks += [v["bit_exact"], v["uniform_pattern"]["bit_exact"]]
                if "oracle" in v:
                    checks.append(v["oracle"]["bit_exact"])
        if not args.no_c5:
            result["c5_mixed"] = c5_mixed(torch, ec, codec, stream, args.c5_gib, args.steps,
                                          args.warmup, args.settle_ms, stage, vthreads)
            checks.append(result["c5_mixed"]["round_trip_bit_exact"])
            if "oracle_bit_exact" in result["c5_mixed"]:
                checks.append(result["c5_mixed"]["oracle_bit_exact"])
        del stage
    if not args.no_verify:
        result["oracle_bit_exact"] = bool(checks) and all(checks)
    if rank == 0:
        if not args.no_cpu:
            log("cpu baseline")
            result["cpu_baseline"] = cpu_baseline(k, m, B, S, args.cpu_seconds, par[:4].cpu().numpy(),
                                                  world)
            result["c1"] = c1_case(torch, ec, codec, stream, world)
        if not args.no_pmc:
            log("counter passes")
            pmc_traffic(args, result, local, world)
            if "rebuild_small" in result:
                pmc_small(args, result, local, world)
        if not args.no_plugin and world == 1:
            log("plugin lines")
            result["plugin"] = plugin_lines()
        if not args.no_sha and world == 1:
            log("sha-256 lines")
            result["sha256"] = sha_lines(torch, codec, stream, data, n, B, cpu_threads(world))
        if args.sweep and world == 1:
            del data, par
            result["sweep"] = sweep(torch, ec, codec, stream, args.sweep_gib, max(3, args.steps // 4),
                                    args.warmup, args.settle_ms, cpu=not args.no_cpu)

    if rank == 0:
        print(json.dumps(result), flush=True)
    codec.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
