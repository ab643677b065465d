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
