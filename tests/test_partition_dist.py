"""Multi-rank path on CPU (gloo, world_size 2): block-index partition is
disjoint and complete, per-rank synthetic inputs equal the single-rank
global batch, and the job time is the max over ranks."""
import json
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, SEED


def test_block_range_covers_exactly():
    from memo_amd.partition import block_range
    for n in [0, 1, 7, 4096, 32768]:
        for w in [1, 2, 3, 4, 8]:
            got = [block_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in got) == n
            pos = 0
            for lo, c in got:
                assert lo == pos
                pos += c
    with pytest.raises(ValueError):
        block_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from memo_amd.partition import block_range, max_over_ranks
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, m, B, n = 4, 2, 3000, 10
    S = O.shard_size(B, k)
    lo, cnt = block_range(n, world, rank)
    data = O.fill_blocks(SEED, lo, cnt, B, k, S)
    par = O.encode(k, m, S, data)
    # gather every rank's parity on rank 0 (test only: the product never does this)
    t = torch.from_numpy(np.ascontiguousarray(par.reshape(-1)))
    bufs = [torch.zeros_like(t) for _ in range(world)]  # equal shares: n % world == 0
    dist.all_gather(bufs, t)
    mx = max_over_ranks(0.5 + rank, dist)
    if rank == 0:
        q.put((mx, [b.numpy() for b in bufs]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_partition_gloo():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    mx, parts = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == 1.5
    from oracle import oracle as O
    k, m, B, n = 4, 2, 3000, 10
    S = O.shard_size(B, k)
    whole = O.encode(k, m, S, O.fill_blocks(SEED, 0, n, B, k, S)).reshape(-1)
    assert np.array_equal(np.concatenate(parts), whole)


def test_launch_local_ranks_env(tmp_path):
    """bench.py's own launcher (no torchrun): N children started together,
    each with its RANK / LOCAL_RANK / WORLD_SIZE and one rendezvous port;
    a failing rank fails the launch."""
    import sys
    from memo_amd.partition import launch_local_ranks
    script = tmp_path / "child.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text(
        "import os, sys\n"
        "e = os.environ\n"
        "open(os.path.join(sys.argv[1], e['RANK']), 'w').write("
        "'%s %s %s %s' % (e['LOCAL_RANK'], e['WORLD_SIZE'], e['MASTER_ADDR'], e['MASTER_PORT']))\n"
        "sys.exit(3 if len(sys.argv) > 2 and sys.argv[2] == e['RANK'] else 0)\n")
    assert launch_local_ranks(str(script), [str(out)], 3) == 0
    got = {f.name: f.read_text().split() for f in out.iterdir()}
    assert sorted(got) == ["0", "1", "2"]
    assert {v[3] for v in got.values()} == {got["0"][3]}
    for r, v in got.items():
        assert v[0] == r and v[1] == "3" and v[2] == "127.0.0.1"
    assert launch_local_ranks(str(script), [str(out)], 2, same_device=True) == 0
    assert all((out / r).read_text().split()[0] == "0" for r in ("0", "1"))
    assert launch_local_ranks(str(script), [str(out), "1"], 2) == 3


def test_bench_assemble_per_rank_fields():
    """The bench line for N ranks: value = all payload / the job wall time,
    per-GPU rates from each rank's own kernel time, node sum over the
    slowest rank, both directions' roofline fractions."""
    import bench
    args = bench.parse(["--gpus", "2", "--blocks", "4096", "--steps", "10"])
    S = 104896
    n, B, K = 4096, 1 << 20, 10

    def row(r, enc_ms, reb_ms):
        return {"rank": r, "device": r, "warmup_steps_run": 40,
                "device_identity": {"pci_bus_id": "0000:%02x:00.0" % (0x11 + r), "uuid": "%032x" % (r + 1)},
                "payload_bytes": n * B * 2 * K, "device_seconds": (enc_ms + reb_ms) * K * 1e-3,
                "encode": bench.kstats([enc_ms] * K, 14 * S * n),
                "rebuild": bench.kstats([reb_ms] * K, 14 * S * n),
                "rebuild_bit_exact": True, "rebuild_kernel": "gf_rebuild_kernel"}
    rows = [row(0, 1.0, 1.1), row(1, 1.05, 1.2)]
    res = bench.assemble(args, 2, rows, 0.05, S)
    assert res["n_gpus"] == 2 and res["config"]["global_blocks"] == 8192
    assert res["value"] == round(2 * n * B * 2 * K / 0.05 / 2**30, 3)
    pg = res["ranks"]["per_gpu"]
    assert [p["rank"] for p in pg] == [0, 1]
    assert pg[0]["GiBs"] == round(n * B * 2 / 2.1e-3 / 2**30, 3)
    assert res["ranks"]["node_sum_GiBs"] == round(2 * n * B * 2 * K / (2.25e-3 * K) / 2**30, 3)
    assert res["roofline"]["kernel_ms_max_over_ranks"] == 1.05
    assert res["roofline"]["frac"] == round(14 * S * n / 1e-3 / 1e9 / 8000, 4)
    assert res["roofline_rebuild"]["kernel"] == "gf_rebuild_kernel"
    assert res["rebuild"]["round_trip_bit_exact"]
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in res
    # every rank's side measurements: rank 0's copy rate and PCIe rate, the
    # node's per-rank list and sum
    e2e = lambda p, q: {"pinned": {"value": p, "bit_exact": True}, "pageable": {"value": q, "bit_exact": True}}
    probe = lambda g: {"GBs": g, "kernel_ms_avg": 1.0, "frac": g / 8000}
    orc = lambda ok: {"C2_encode": {"blocks": n, "bytes_compared": n * 4 * S, "bit_exact": ok, "seconds": 0.5},
                      "C3_rebuild": {"blocks": n, "erasures": 4, "bytes_compared": n * 4 * S,
                                     "bit_exact": True, "seconds": 0.7}}
    extras = [{"probe": probe(6400.0), "oracle": orc(True), "e2e": e2e(48.0, 45.0),
               "lat": {"encode_4096B_us": 20.0}},
              {"probe": probe(6300.0), "oracle": orc(False), "e2e": e2e(47.0, 44.0),
               "lat": {"encode_4096B_us": 21.0}}]
    bench.merge_extras(res, extras)
    assert res["roofline"]["achievable"]["GBs"] == 6400.0
    assert res["roofline"]["frac_of_achievable"] == round(res["roofline"]["achieved"] / 6400.0, 4)
    assert res["roofline_rebuild"]["frac_of_achievable"] == round(res["roofline_rebuild"]["achieved"] / 6400.0, 4)
    assert res["roofline"]["achievable_per_rank_GBs"] == [6400.0, 6300.0]
    # a rank whose batch differs from the oracle fails the whole check
    assert res["oracle_parity"]["C2_encode"]["bit_exact"] is False
    assert res["oracle_parity"]["C2_encode"]["blocks"] == 2 * n
    assert res["oracle_parity"]["C3_rebuild"]["bit_exact"] is True
    assert [p["pci_bus_id"] for p in res["ranks"]["per_gpu"]] == ["0000:11:00.0", "0000:12:00.0"]
    assert res["ranks"]["distinct_devices"] == 2
    # the same rows naming one GPU twice: no line (unless --same-device)
    dup = [dict(r) for r in rows]
    dup[1]["device_identity"] = dict(dup[0]["device_identity"])
    with pytest.raises(RuntimeError, match="same GPU"):
        bench.assemble(args, 2, dup, 0.05, S)
    same = bench.parse(["--gpus", "2", "--same-device", "--blocks", "4096", "--steps", "10"])
    assert bench.assemble(same, 2, dup, 0.05, S)["ranks"]["distinct_devices"] == 1
    assert res["end_to_end"]["pinned"]["value"] == 48.0
    assert res["end_to_end"]["node_sum"] == {"pinned": 95.0, "pageable": 89.0}
    assert [x["rank"] for x in res["end_to_end"]["per_rank"]] == [0, 1]
    assert res["host_call_latency"]["encode_4096B_us"] == 20.0


def test_bench_assemble_world_8_c4_line():
    """The first 8-GPU line (C4) is self-describing: eight ranks with
    distinct device identities give distinct_devices 8, 32768 global blocks
    (4096 per GPU), and the line names the N = 1-only legs it left out."""
    import bench
    args = bench.parse(["--gpus", "8", "--steps", "10"])
    S = 104896
    n, B, K = args.blocks, args.block_bytes, 10
    assert (n, B) == (4096, 1 << 20)
    rows = [{"rank": r, "device": r, "warmup_steps_run": 40,
             "device_identity": {"pci_bus_id": "0000:%02x:00.0" % (0x05 + 0x10 * r), "uuid": "%032x" % (0xa0 + r)},
             "payload_bytes": n * B * 2 * K, "device_seconds": 2.0e-3 * K,
             "encode": bench.kstats([0.98] * K, 14 * S * n), "rebuild": bench.kstats([1.0] * K, 14 * S * n),
             "rebuild_bit_exact": True, "rebuild_kernel": "decode + gf_mac_kernel"} for r in range(8)]
    res = bench.assemble(args, 8, rows, 0.021, S)
    assert res["n_gpus"] == 8 and res["scaling"] == "weak"
    assert res["ranks"]["distinct_devices"] == 8
    assert res["config"]["global_blocks"] == 32768 and res["config"]["blocks_per_gpu"] == 4096
    assert "C4 at N=8" in res["config"]["workload"]
    assert len(res["ranks"]["per_gpu"]) == 8
    assert set(res["skipped_at_n"]) == {"rebuild_small", "c5_mixed", "plugin", "sha256"}
    assert res["value"] == round(8 * n * B * 2 * K / 0.021 / 2**30, 3)
    # flags that turn a leg off leave it out of the list; N = 1 lists none
    quiet = bench.parse(["--gpus", "8", "--no-plugin", "--no-sha", "--sweep"])
    assert set(bench.skipped_at_n(quiet, 8)) == {"rebuild_small", "c5_mixed", "sweep"}
    one = bench.parse(["--gpus", "1"])
    assert bench.skipped_at_n(one, 1) == {}
    assert "skipped_at_n" not in bench.assemble(one, 1, rows[:1], 0.002, S)
    # two ranks on one device are refused in an 8-rank line too
    dup = [dict(r) for r in rows]
    dup[7]["device_identity"] = dict(dup[3]["device_identity"])
    with pytest.raises(RuntimeError, match="same GPU"):
        bench.assemble(args, 8, dup, 0.021, S)


def test_world_8_line_fits_the_rank_lease(monkeypatch):
    """The 8-GPU line (C4) with the job's CPU share split 8 ways (16 CPUs:
    2 threads per rank) still fits --rank-timeout: the whole-batch oracle
    checks of every rank's own 4096 x 1 MiB C2 / C3 batches, the CPU
    baseline and the counter passes on rank 0 -- estimated from the rates
    measured on the GPU boxes (bench.POST_RATES) -- plus the timed steps;
    and assemble() turns the eight rows into the line."""
    import bench
    monkeypatch.setattr(bench, "host_cores", lambda: 256)
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: 16)
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    args = bench.parse(["--gpus", "8"])
    world, S = 8, 104896
    per_rank = max(1, bench.cpu_threads(world) // world)   # what main() gives each rank's checks
    assert per_rank == 2
    est = bench.post_timed_seconds(args, world, per_rank, S)
    timed = (args.warmup + args.steps) * 2.0e-3 + args.settle_ms * 1e-3
    assert est["rank0"] + timed < args.rank_timeout, est
    assert est["rank"] <= est["rank0"]
    assert set(est["legs"]) >= {"oracle_checks", "cpu_baseline", "counter_passes"}
    assert not {"rebuild_small", "c5_mixed", "plugin", "sha256"} & set(est["legs"])
    # one thread per rank (a 8-CPU share) still fits; the N = 1 line, with
    # every leg, fits its own lease on the box's 16 threads
    assert bench.post_timed_seconds(args, world, 1, S)["rank0"] + timed < args.rank_timeout
    one = bench.parse(["--gpus", "1"])
    assert bench.post_timed_seconds(one, 1, 16, S)["rank0"] + timed < one.rank_timeout
    # a slower box (half the rates, twice the pass times) still fits at N = 8
    slow = {k: (v / 2 if k.endswith("GiBs") else v * 2) for k, v in bench.POST_RATES.items()}
    assert bench.post_timed_seconds(args, world, per_rank, S, slow)["rank0"] + timed < args.rank_timeout
    rows = [{"rank": r, "device": r, "warmup_steps_run": 40,
             "device_identity": {"pci_bus_id": "0000:%02x:00.0" % (0x05 + 0x10 * r), "uuid": "%032x" % (0xa0 + r)},
             "payload_bytes": args.blocks * args.block_bytes * 2 * args.steps,
             "device_seconds": 2.0e-3 * args.steps,
             "encode": bench.kstats([0.98] * args.steps, 14 * S * args.blocks),
             "rebuild": bench.kstats([1.0] * args.steps, 14 * S * args.blocks),
             "rebuild_bit_exact": True, "rebuild_kernel": "gf_mac_images_kernel"} for r in range(world)]
    res = bench.assemble(args, world, rows, 2.0e-3 * args.steps, S)
    assert res["n_gpus"] == 8 and res["ranks"]["distinct_devices"] == 8


def test_cpu_share_is_bounded(monkeypatch):
    """The CPU baseline's threads: at N = 1 the affinity set capped by the
    cgroup quota and OMP_NUM_THREADS; at N > 1 the job's node share (the
    quota), not one rank's share -- OMP_NUM_THREADS=1, which
    torch.distributed.run sets for every rank, is not a share."""
    import bench
    assert 1 <= bench.cpu_share() <= bench.host_cores()
    assert bench.cpu_threads() == bench.cpu_share()
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_share() <= 3 and bench.cpu_threads(1) <= 3
    monkeypatch.setattr(bench, "host_cores", lambda: 256)
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: 128)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.cpu_threads(1) == 1
    assert bench.cpu_threads(8) == 128          # the quota, all 8 ranks' share
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.cpu_threads(1) == 16
    assert bench.cpu_threads(4) == 64           # 16 per GPU x 4 ranks, under the quota
    assert bench.cpu_threads(8) == 128
    monkeypatch.setattr(bench, "_cgroup_cpus", lambda: None)
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_threads(8) == 256


def test_duplicate_devices_refused():
    """A multi-rank line whose ranks report the same GPU (PCI bus id or
    UUID) is refused unless the run asked for one shared device."""
    import bench
    ident = lambda bus, uid: {"pci_bus_id": bus, "uuid": uid}
    rows = [{"rank": 0, "device_identity": ident("0000:11:00.0", "a" * 32)},
            {"rank": 1, "device_identity": ident("0000:11:00.0", "b" * 32)}]
    with pytest.raises(RuntimeError, match="same GPU"):
        bench.check_devices(rows, same_device=False)
    rows[1]["device_identity"] = ident("0000:12:00.0", "a" * 32)
    with pytest.raises(RuntimeError, match="uuid"):
        bench.check_devices(rows, same_device=False)
    bench.check_devices(rows, same_device=True)
    rows[1]["device_identity"] = ident("0000:12:00.0", "b" * 32)
    bench.check_devices(rows, same_device=False)
    with pytest.raises(RuntimeError, match="no device identity"):
        bench.check_devices([rows[0], {"rank": 1}], same_device=False)


def test_launcher_kills_a_hung_rank(tmp_path):
    """bench.py's own launcher bounds the run: a rank that never finishes is
    killed (by PID) after the timeout, the others too, and the launch
    returns non-zero well before a driver limit would."""
    import sys
    import time
    from memo_amd.partition import launch_local_ranks
    script = tmp_path / "child.py"
    script.write_text("import os, time\n"
                      "time.sleep(3600 if os.environ['RANK'] == '1' else 0)\n")
    t0 = time.monotonic()
    rc = launch_local_ranks(str(script), [], 2, timeout=3)
    assert rc != 0 and time.monotonic() - t0 < 30


def _bench_json(r):
    import json
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    # stdout is exactly rank 0's JSON line (gloo's connect messages go to
    # stderr), as the driver reads it
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    return json.loads(lines[0])


BENCH_SMALL = ["--gpus", "2", "--same-device", "--steps", "3", "--warmup", "2", "--settle-ms", "0",
               "--blocks", "64", "--no-cpu", "--no-e2e", "--no-small", "--no-pmc"]


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_launches_its_own_ranks(ranks):
    """`python bench.py --gpus N` with no external launcher starts the N ranks
    itself (all on cuda:0 here; one per GPU on a node), each encoding and
    rebuilding its own 64 blocks; rank 0 prints one line."""
    import subprocess
    import sys
    args = list(BENCH_SMALL)
    args[args.index("--gpus") + 1] = str(ranks)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    res = _bench_json(r)
    assert res["n_gpus"] == ranks and res["config"]["global_blocks"] == 64 * ranks
    assert res["value"] > 0 and res["rebuild"]["round_trip_bit_exact"]
    assert [p["rank"] for p in res["ranks"]["per_gpu"]] == list(range(ranks))
    assert res["ranks"]["node_sum_GiBs"] > 0


@pytest.mark.gpu
def test_bench_two_ranks_under_torchrun():
    """The driver's N>1 launch: torch.distributed.run starts the ranks, and
    bench.py uses them (gloo for the barrier/max, no RCCL)."""
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py")] + BENCH_SMALL
    res = _bench_json(subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT))
    assert res["n_gpus"] == 2 and res["config"]["global_blocks"] == 128
    assert res["value"] > 0 and res["rebuild"]["round_trip_bit_exact"]


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_n2_line_is_self_sufficient():
    """At N = 2 the line still carries the CPU baseline (rank 0, after the
    timed steps), every rank's PCIe end-to-end rate and their sum, the
    counter-measured traffic of this run, and the loaded library's build id
    (== the sources' hash)."""
    import subprocess
    import sys
    args = ["--gpus", "2", "--same-device", "--steps", "3", "--warmup", "2", "--settle-ms", "0",
            "--blocks", "256", "--no-small", "--cpu-seconds", "1"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=380, cwd=ROOT)
    res = _bench_json(r)
    assert res["n_gpus"] == 2
    cb = res["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["bit_exact_vs_gpu"]
    assert cb["n_gpus"] == 2 and cb["per_gpu_share"] == round(cb["cores"] / 2, 2)
    # every rank compared its whole batch with the CPU oracle
    assert res["oracle_bit_exact"] and res["oracle_parity"]["C2_encode"]["ranks"] == 2
    assert res["oracle_parity"]["C2_encode"]["blocks"] == 512
    assert res["oracle_parity"]["C3_rebuild"]["bit_exact"]
    # (both ranks share one GPU here: the probe and the kernels contend, so
    # only the presence of the achievable figure is checked)
    assert res["roofline"]["frac_of_achievable"] > 0
    assert len(res["end_to_end"]["per_rank"]) == 2 and res["end_to_end"]["node_sum"]["pinned"] > 0
    assert res["end_to_end"]["pinned"]["bit_exact"]
    assert res["roofline"]["traffic"] > 0 and res["roofline"]["traffic_ratio"] < 1.5, res["roofline"]
    assert res["roofline_rebuild"]["traffic"] > 0
    assert res["build_matches_sources"]
    # the N = 1-only legs it left out are named in the line
    assert set(res["skipped_at_n"]) == {"c5_mixed", "plugin", "sha256"}


def _fake_rocprof(monkeypatch, rows_by_counter):
    """subprocess.run stand-in for the bench's rocprofv3 child runs: writes
    a counter_collection.csv with the given rows into the -d directory."""
    import csv
    import subprocess

    class R:
        returncode = 0
        stderr = b""

    def run(cmd, **kw):
        d = cmd[cmd.index("-d") + 1]
        os.makedirs(os.path.join(d, "host"), exist_ok=True)
        pmc = cmd[cmd.index("--pmc") + 1:cmd.index("-d")]
        with open(os.path.join(d, "host", "x_counter_collection.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value",
                                              "Start_Timestamp", "End_Timestamp"])
            w.writeheader()
            for r in rows_by_counter:
                if r["Counter_Name"] in pmc:
                    w.writerow(r)
        return R()
    monkeypatch.setattr(subprocess, "run", run)


def test_counter_passes_fold_into_the_line(monkeypatch):
    """pmc_traffic and pmc_small (run after the timed steps as rocprofv3
    child processes) parse the counter files into roofline.traffic and the
    4 KiB lines' counters; a failed pass leaves a note, never a crash."""
    import bench
    args = bench.parse(["--gpus", "1"])
    S, n = 104896, 4096
    enc = "void memo_ec::gf_mac_kernel<10, 4, true, false>(memo_ec::MacLaunch)"
    reb = "void memo_ec::gf_mac_kernel<10, 4, true, true>(memo_ec::MacLaunch)"
    rows = []
    for disp, name, fetch, write in [(1, enc, 2.9e6, 1.7e6), (2, reb, 2.95e6, 1.7e6)]:
        rows += [{"Dispatch_Id": disp, "Kernel_Name": name, "Counter_Name": "FETCH_SIZE",
                  "Counter_Value": fetch, "Start_Timestamp": 0, "End_Timestamp": 1},
                 {"Dispatch_Id": disp, "Kernel_Name": name, "Counter_Name": "WRITE_SIZE",
                  "Counter_Value": write, "Start_Timestamp": 0, "End_Timestamp": 1}]
    k16e = "void memo_ec::gf_mac_kernel<16, 4, true, false>(memo_ec::MacLaunch)"
    k16r = "void memo_ec::gf_mac_kernel<16, 4, true, true>(memo_ec::MacLaunch)"
    dec = "void memo_ec::decode_rows_k_kernel<16, 4>(memo_ec::DecodeLaunch)"
    for disp, name in [(10, k16e), (11, dec), (12, k16r)]:
        for c, v in [("SQ_INSTS_VALU", 4.3e8), ("SQ_INSTS_SALU", 2.2e7), ("SQ_INSTS_LDS", 2.6e7),
                     ("SQ_WAVES", 262144), ("SQ_ACTIVE_INST_ANY", 4.9e8), ("SQ_WAIT_INST_ANY", 4.6e8),
                     ("SQ_WAIT_ANY", 2.8e8), ("SQ_WAVE_CYCLES", 1.38e9), ("GRBM_GUI_ACTIVE", 1.57e7)]:
            rows.append({"Dispatch_Id": disp, "Kernel_Name": name, "Counter_Name": c, "Counter_Value": v,
                         "Start_Timestamp": 1000, "End_Timestamp": 1000 + 906000})
    _fake_rocprof(monkeypatch, rows)
    res = {"build_id": "x" * 64,
           "roofline": {"bytes_per_launch": 14 * S * n}, "roofline_rebuild": {"bytes_per_launch": 14 * S * n},
           "rebuild_small": {"RS(16,4)": {"frac": 0.65}, "RS(10,4)": {"frac": 0.71}}}
    bench.pmc_traffic(args, res, 0, 1)
    assert res["roofline"]["traffic"] == int(round((2 * 2.9e6 + 1.7e6) * 1024))
    assert res["roofline_rebuild"]["traffic"] > 0 and "traffic_source" in res["roofline_rebuild"]
    bench.pmc_small(args, res, 0, 1)
    c = res["rebuild_small"]["RS(16,4)"]["counters"]
    assert set(c) == {"encode MAC", "rebuild MAC", "decode rows"}
    assert c["rebuild MAC"]["valu_busy"] == round(4.3e8 * 2 / (1024 * 1.57e7 / 8), 4)
    assert c["encode MAC"]["clock_GHz"] == round(1.57e7 / 8 / 906000, 3)
    assert c["encode MAC"]["valu_per_wave"] == round(4.3e8 / 262144, 1)
    assert "counters_source" in res["rebuild_small"]
    # a pass that produces nothing: a note in the line, no exception
    _fake_rocprof(monkeypatch, [])
    res2 = {"build_id": "x" * 64, "roofline": {"bytes_per_launch": 1}, "rebuild_small": {"RS(16,4)": {}}}
    bench.pmc_small(args, res2, 0, 1)
    assert "counters_note" in res2["rebuild_small"]
    bench.pmc_traffic(args, res2, 0, 1)
    assert res2["roofline"]["traffic"] is None and "traffic_note" in res2["roofline"]


def test_whole_batch_checks_catch_one_byte():
    """verify_encode / verify_rebuild (the bench line's whole-batch oracle
    comparison) stream a batch through small staging chunks and report one
    flipped byte anywhere in it (CPU tensors stand in for device ones)."""
    import torch
    import bench
    from oracle import oracle as O
    k, m, B, n, e = 4, 2, 5000, 37, 2
    S = O.shard_size(B, k)
    data = O.fill_blocks(SEED, 0, n, B, k, S)
    par = O.encode(k, m, S, data)
    stage = bench.HostStage(torch, chunk_bytes=5 * (k + m) * S)  # several chunks
    d, p = torch.from_numpy(data.copy()), torch.from_numpy(par.copy())
    assert bench.verify_encode(stage, k, m, S, d, p, 2)["bit_exact"]
    p[n - 1, m * S - 1] ^= 1
    v = bench.verify_encode(stage, k, m, S, d, p, 2)
    assert not v["bit_exact"] and v["blocks"] == n and v["bytes_compared"] == n * m * S
    s_idx, l_idx = O.erasures(SEED, 0, n, k, m, e)
    surv = torch.from_numpy(O.gather(k, m, S, data, par, s_idx))
    out = torch.from_numpy(O.gather(k, m, S, data, par, l_idx))
    assert bench.verify_rebuild(stage, k, m, S, s_idx, surv, l_idx, out, 2)["bit_exact"]
    out[17, 5] ^= 0x80
    assert not bench.verify_rebuild(stage, k, m, S, s_idx, surv, l_idx, out, 2)["bit_exact"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_default_line_runs_every_leg():
    """The driver's own command shape at N = 1 (fewer steps, a short CPU
    sample): the line carries the whole-batch oracle comparison of C2, C3,
    the 4 KiB rebuilds and C5, the achievable-rate probe, the 4 KiB counter
    summary, counter traffic, the CPU baseline, the device identity, the
    SHA-256 lines and the plugin-level lines."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "5",
                        "--warmup", "2", "--cpu-seconds", "1"],
                       capture_output=True, text=True, timeout=560, cwd=ROOT)
    res = _bench_json(r)
    assert res["oracle_bit_exact"] is True
    assert set(res["oracle_parity"]) == {"C2_encode", "C3_rebuild"}
    for name in ("RS(10,4)", "RS(16,4)"):
        sm = res["rebuild_small"][name]
        assert sm["oracle"]["bit_exact"] and sm["uniform_pattern"]["bit_exact"]
        assert 0 < sm["frac_of_achievable"] <= 1.05
        assert set(sm["counters"]) == {"encode MAC", "rebuild MAC", "decode rows"}, res["rebuild_small"]
    assert res["c5_mixed"]["oracle_bit_exact"] and len(res["c5_mixed"]["groups"]) == 12
    assert 0 < res["roofline"]["frac_of_achievable"] <= 1.05  # probe timing noise: a few %
    assert res["roofline"]["traffic_ratio"] < 1.1
    assert res["cpu_baseline"]["bit_exact_vs_gpu"] and res["c1"]["bit_exact"]
    assert res["c1"]["encode"]["cpu_simd_ms"] > 0 and res["c1"]["rebuild_e2"]["cpu_simd_ms"] > 0
    assert "skipped_at_n" not in res
    assert res["ranks"]["per_gpu"][0]["uuid"] and res["build_matches_sources"]
    for key in ("C2 batch, 1 MiB blocks", "4 KiB blocks"):
        assert res["sha256"][key]["bit_exact"] and res["sha256"][key]["checked"] >= 4096, res["sha256"]
    for key, pl in res["plugin"].items():
        assert pl["ok"] and pl["erasure"]["fetch_after_repair_ok"], (key, pl)
        assert pl["erasure"]["unrecoverable"] == 0 and pl["erasure"]["degraded_codec_calls"] >= 1


def test_plugin_lines_parse_and_flag_failures(tmp_path):
    """bench.py's plugin leg on a stand-in binary (no GPU): a clean run is
    kept whole, a non-zero exit or a missing rate marks the row not ok with
    the child's stderr, and a missing binary is a note, not a crash."""
    import bench
    line = json.dumps({"workload": "x", "reps": 5,
                       "erasure": {k: [1.0, 3.0, 2.0, 5.0, 4.0] for k in bench.PLUGIN_KEYS} | {
                           "fetch_after_repair_ok": True, "unrecoverable": 0},
                       "replication": {"store_GiBs": [2.0, 2.0, 2.0, 2.0, 2.0],
                                       "fetch_GiBs": [1.0, 1.0, 4.0, 1.0, 1.0]},
                       "replication_unvalidated": {"store_GiBs": [4.0, 4.0, 4.0, 4.0, 4.0],
                                                   "fetch_GiBs": [1.0, 1.0, 1.0, 1.0, 1.0]}})
    fake = tmp_path / "bench_plugin"
    fake.write_text("#!/bin/sh\n[ \"$1\" = 3 ] && { echo oops >&2; echo '%s'; exit 1; }\n"
                    "[ \"$1\" = 5 ] && { echo '{\"erasure\": {}}'; exit 0; }\n"
                    "[ \"$3\" = 5 ] || exit 9\necho '%s'\n" % (line, line))
    fake.chmod(0o755)
    out = bench.plugin_lines(str(fake), [(2, 4096), (3, 4096), (5, 64)], timeout=30)
    row = out["2x4096"]
    assert row["ok"] and row["erasure"]["fetch_after_repair_ok"] and row["reps"] == 5
    # {median, min, max, n} per rate, from the five repetitions
    st = row["erasure"]["store_GiBs"]
    assert (st["median"], st["min"], st["max"], st["n"]) == (3.0, 1.0, 5.0, 5)
    assert st["samples"] == [1.0, 3.0, 2.0, 5.0, 4.0]
    assert row["replication"]["fetch_GiBs"]["median"] == 1.0
    assert row["replication"]["fetch_GiBs"]["max"] == 4.0
    # ratios per repetition (erasure / replication of the same repetition)
    assert row["ratio"]["store"]["samples"] == [0.5, 1.5, 1.0, 2.5, 2.0]
    assert row["ratio"]["store"]["median"] == 1.5
    assert row["ratio"]["fetch"]["samples"] == [1.0, 3.0, 0.5, 5.0, 4.0]
    assert row["ratio"]["fetch"]["median"] == 3.0 and row["ratio"]["fetch"]["min"] == 0.5
    # the same against replication through plain peers
    assert row["replication_unvalidated"]["store_GiBs"]["median"] == 4.0
    assert row["ratio_unvalidated"]["store"]["samples"] == [0.25, 0.75, 0.5, 1.25, 1.0]
    assert row["ratio_unvalidated"]["fetch"]["median"] == 3.0
    assert not out["3x4096"]["ok"] and "oops" in out["3x4096"]["note"]
    assert not out["5x64"]["ok"]
    gone = bench.plugin_lines(str(tmp_path / "missing"), [(1, 1)], timeout=30)
    assert not gone["1x1"]["ok"] and gone["1x1"]["note"]


def test_sha_digest_check_catches_one_flipped_byte():
    """bench.py's hashlib check of GPU digests (no GPU: digests made here)."""
    import hashlib
    import bench
    rng = np.random.default_rng(SEED)
    msgs = rng.integers(0, 256, size=(40, 300), dtype=np.uint8)
    digs = np.stack([np.frombuffer(hashlib.sha256(bytes(64) + m[:257].tobytes()).digest(), np.uint8)
                     for m in msgs])
    assert bench.sha_digests_ok(msgs, digs, range(40), 257, 4)
    digs[17, 3] ^= 1
    assert not bench.sha_digests_ok(msgs, digs, range(40), 257, 4)
    assert bench.sha_digests_ok(msgs, digs, range(17), 257, 1)
