"""GPU: a native program drives a round through the C ABI alone
(examples/c_abi_round.cpp — no Python, no torch in the process) and checks
it bit-for-bit against a host restatement of the reference order."""
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_native_c_abi_round():
    exe = os.path.join(ROOT, "examples", "c_abi_round")
    if not os.path.exists(exe):
        pytest.fail("examples/c_abi_round not built (run __graft_entry__.build())")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK:" in r.stdout and "gfx950" in r.stdout, r.stdout
