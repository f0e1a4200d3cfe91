"""The C-ABI from a plain C program (tests/c/abi_test.c): what a cgo
binding sees -- include/uplink_ec.h + libuplink_ec.so with host buffers, no
Python or torch in the process -- checked against the CPU oracle."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c", "build", "abi_test")
BIN_CHECKED = os.path.join(HERE, "c", "build", "abi_test_checked")


def test_c_client_links_against_the_library():
    if not os.path.exists(BIN):
        pytest.skip("tests/c not built (run __graft_entry__.build())")
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, timeout=60).stdout
    assert "libuplink_ec.so" in out and "not found" not in out


@pytest.mark.gpu
def test_c_client_on_gpu():
    assert os.path.exists(BIN), "tests/c/build/abi_test missing: build() compiles it"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1].startswith("ok")


@pytest.mark.gpu
def test_c_client_on_gpu_checked_library():
    """The same client against libuplink_ec_checked.so, whose stripe kernels
    compare every global address with the launch's declared byte ranges and
    trap (with the site printed) on one outside them."""
    assert os.path.exists(BIN_CHECKED), "tests/c/build/abi_test_checked missing: build() compiles it"
    r = subprocess.run([BIN_CHECKED], capture_output=True, text=True, timeout=120)
    assert "uplink_ec checked" not in r.stdout + r.stderr, r.stdout + r.stderr
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1].startswith("ok")
