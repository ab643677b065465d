"""The C++ erasure plugin (host/): the reference's redundancy-path semantics
tests ported in host/tests/test_erasure.cc (CHB round trip, missing_block,
CHB_no_peer, availability, evict/repair, CHB_unavailable; silo contract).
CPU: build + the tests that need no codec.  GPU: every test, codec on the
MI355X through libmemo_ec.so."""
import os
import subprocess

import pytest

from conftest import ROOT

HOST = os.path.join(ROOT, "host")
BIN = os.path.join(HOST, "_build", "test_erasure")


def _build():
    subprocess.check_call(["make", "-s", "-j4", "-C", HOST])
    assert os.path.exists(BIN)


def _run(*args, timeout=600):
    r = subprocess.run([BIN, *args], capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-4000:], r.stderr[-4000:])
    return r


def test_plugin_builds_and_cpu_tests_pass():
    _build()
    r = _run("--cpu-only")
    assert r.returncode == 0, r.stderr
    assert " 0 failed" in r.stdout


def test_plugin_surface_matches_reference_consensus():
    """host/tests/surface_check.cc static_asserts that ErasureConsensus
    declares every Consensus virtual of the reference (Consensus.hh:24-142)
    with its exact signature (_store, both _fetch, _remove, _resign, stat,
    make_local, redundancy, stats; make_remote through StackedConsensus)."""
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I" + os.path.join(ROOT, "include"),
                        os.path.join(HOST, "tests", "surface_check.cc")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]


def test_integration_class_matches_plugin_overrides():
    """INTEGRATION.md's Erasure class overrides the same Consensus members as
    host/erasure_consensus.hh's ErasureConsensus (the drop-in a maintainer
    adds is the code that is tested, up to namespaces and elle types)."""
    import re

    def overrides(text):
        text = re.sub(r"//[^\n]*", "", text)
        names = set()
        for m in re.finditer(r"(\w+)\s*\([^;{]*\)\s*(?:const\s*)?override", text):
            if not m.group(1)[0].isupper():  # not the destructor
                names.add(m.group(1))
        return names

    with open(os.path.join(HOST, "erasure_consensus.hh")) as f:
        hh = f.read()
    cls = hh[hh.index("class ErasureConsensus"):]
    cls = cls[:cls.index("\n};")]
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    dcls = doc[doc.index("class Erasure : public StackedConsensus"):]
    dcls = dcls[:dcls.index("\n};")]
    want = {"_store", "_fetch", "_remove", "_resign", "stat", "make_local", "redundancy", "stats"}
    assert overrides(cls) == want, overrides(cls)
    assert overrides(dcls) == want, overrides(dcls)
    # boost::optional<boost::asio::ip::address> as the reference declares it
    assert "boost::optional<boost::asio::ip::address> listen_address" in dcls


def test_plugin_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    _build()
    r = _run("CHB")
    assert r.returncode != 0
    assert "no such GPU" in r.stderr


@pytest.mark.gpu
def test_plugin_semantics_on_gpu():
    _build()
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout


@pytest.mark.gpu
def test_plugin_bench_round_trip_on_gpu():
    """host/tests/bench_plugin.cc end to end at a small size: store, healthy
    and degraded multi-fetch, repair after eviction, against replication;
    it exits non-zero if any block comes back wrong or is unrecoverable."""
    import json
    _build()
    r = subprocess.run([os.path.join(HOST, "_build", "bench_plugin"), "96", "70000", "2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["erasure"]["fetch_ok"] and d["erasure"]["degraded_ok"]
    assert d["erasure"]["repaired_blocks"] > 0 and d["erasure"]["unrecoverable"] == 0
    assert d["erasure"]["degraded_codec_calls"] >= 1
    # two interleaved repetitions, one rate per repetition
    assert d["reps"] == 2 and len(d["erasure"]["store_GiBs"]) == 2 and len(d["replication"]["fetch_GiBs"]) == 2
