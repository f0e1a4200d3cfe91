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


def _run_client(binary, cache_dir, timeout=120):
    """Run a C client in the environment an integrator gets by default --
    run-time encoder compilation on, an empty disk cache -- with the library's
    diagnostic log on (UPLINK_EC_LOG: every run-time compile and module load
    with its duration).  Its RS(10,20) per-stripe calls must not start a hiprtc
    compile (the library starts one only for whole-segment launches), so the
    process exits in seconds instead of waiting for one at exit (the checked
    client's round-2, round-4 and round-5 timeouts).  On a
    timeout, fail with everything it printed so far: the client stamps each
    phase, so the last line names where it stopped."""
    env = dict(os.environ, UPLINK_EC_LOG="1", UPLINK_EC_JIT_CACHE=str(cache_dir))
    env.pop("UPLINK_EC_JIT", None)
    try:
        return subprocess.run([binary], capture_output=True, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired as e:
        out = (e.stdout or b"").decode() if isinstance(e.stdout, bytes) else (e.stdout or "")
        err = (e.stderr or b"").decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        pytest.fail(f"{os.path.basename(binary)} timed out after {timeout} s; its output:\n{out}\n{err}")


def _no_compile_started(r):
    log = r.stdout + r.stderr
    assert "encoder: start" not in log and "joining 1 encoder compile" not in log, log


@pytest.mark.gpu
def test_c_client_on_gpu(tmp_path):
    assert os.path.exists(BIN), "tests/c/build/abi_test missing: build() compiles it"
    r = _run_client(BIN, tmp_path / "jit")
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1].startswith("ok")
    _no_compile_started(r)


@pytest.mark.gpu
def test_c_client_on_gpu_checked_library(tmp_path):
    """The same client against libuplink_ec_checked.so, whose stripe kernels
    compare every global address with the launch's declared byte ranges and
    trap (with the site printed) on one outside them.  First, before any GPU
    work, the two libraries must be one build (ec_build_id): a stale checked
    library is reported as such instead of running."""
    assert os.path.exists(BIN_CHECKED), "tests/c/build/abi_test_checked missing: build() compiles it"
    ids = [subprocess.run([b, "--build-id"], capture_output=True, text=True, timeout=30).stdout.strip()
           for b in (BIN, BIN_CHECKED)]
    assert ids[0] and ids[0] == ids[1], f"checked library build {ids[1]} is not the product's {ids[0]}: rebuild both"
    r = _run_client(BIN_CHECKED, tmp_path / "jit")
    assert "uplink_ec checked" not in r.stdout + r.stderr, r.stdout + r.stderr
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1].startswith("ok")
    _no_compile_started(r)


BIN_EXIT = os.path.join(HERE, "c", "build", "exit_test")


@pytest.mark.gpu
def test_exit_while_encoder_compiles(tmp_path):
    """main() returns while hiprtc compiles RS(11,23)'s encoder in the library's
    background thread (tests/c/exit_test.c): exit waits for the
    compile before the compiler library's destructors run, so the process
    exits 0 with nothing on stderr (round 2: "double free or corruption")."""
    assert os.path.exists(BIN_EXIT), "tests/c/build/exit_test missing: build() compiles it"
    env = dict(os.environ, UPLINK_EC_JIT_CACHE=str(tmp_path / "jit"))
    r = subprocess.run([BIN_EXIT, "11", "23"], capture_output=True, text=True, timeout=300, env=env)
    # libdrm's note about its ids file is the driver stack's, not the library's
    err = [ln for ln in r.stderr.splitlines() if "amdgpu.ids" not in ln]
    assert r.returncode == 0 and not err, (r.returncode, r.stdout, r.stderr)
    assert "while RS(11,23)'s encoder compiles" in r.stdout
    # the compile that exit waited for finished and published its code object
    cached = sorted(p.name for p in (tmp_path / "jit").iterdir())
    assert any(n.endswith(".co") for n in cached) and any(n.endswith(".names") for n in cached), cached
    assert (tmp_path / "jit").stat().st_mode & 0o077 == 0


@pytest.mark.gpu
def test_jit_cache_entry_with_a_bad_digest_is_recompiled(tmp_path):
    """A cached code object that does not match the digest in its .names file
    is removed and compiled again (the cache's code runs on the GPU)."""
    env = dict(os.environ, UPLINK_EC_JIT_CACHE=str(tmp_path / "jit"))
    r = subprocess.run([BIN_EXIT, "11", "23"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    co = [p for p in (tmp_path / "jit").iterdir() if p.name.endswith(".co")]
    assert len(co) == 1
    data = bytearray(co[0].read_bytes())
    data[len(data) // 2] ^= 0xFF
    co[0].write_bytes(bytes(data))
    # the damaged entry is not used: the encoder is compiled again, so it is not ready
    # at once and the client sees a compile in progress (exit_test's own check)
    r = subprocess.run([BIN_EXIT, "11", "23"], capture_output=True, text=True, timeout=300, env=env)
    err = [ln for ln in r.stderr.splitlines() if "amdgpu.ids" not in ln]
    assert r.returncode == 0 and not err, (r.returncode, r.stdout, r.stderr)
    assert co[0].read_bytes() != bytes(data), "the damaged code object was not replaced"
