"""The library's host code (snappy framing, ECIES, one-pass decrypt+unsnap,
the file header parser) under AddressSanitizer + UndefinedBehaviorSanitizer:
tests/host_fuzz.cpp feeds it valid inputs and seeded mutations of them and
checks that every call fails with a status or returns the original bytes.
CPU only (host code; GPU sanitizers are not available on this pool)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def fuzzer(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = tmp_path_factory.mktemp("asan") / "host_fuzz"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", str(ROOT / "tests" / "host_fuzz.cpp"),
           str(ROOT / "carbonado_amd" / "csrc" / "host_snap.cpp"),
           str(ROOT / "carbonado_amd" / "csrc" / "host_stages.cpp"),
           str(ROOT / "carbonado_amd" / "csrc" / "host_stages_par.cpp"),
           str(ROOT / "carbonado_amd" / "csrc" / "gcm_vaes.cpp"),
           str(ROOT / "carbonado_amd" / "csrc" / "file_container.cpp"), "-I" + str(ROOT / "include"),
           "-lcrypto", "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe


@pytest.mark.parametrize("seed,gcm", [("0xF022", "vaes"), ("0xBEEF", "vaes"), ("0xF022", "openssl")])
def test_host_code_under_asan_ubsan(fuzzer, seed, gcm):
    env = dict(os.environ, CHIP_GCM=gcm, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(fuzzer), "6", seed], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout


@pytest.fixture(scope="module")
def tsan_fuzzer(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = tmp_path_factory.mktemp("tsan") / "host_fuzz"
    src = ROOT / "carbonado_amd" / "csrc"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", str(ROOT / "tests" / "host_fuzz.cpp"),
           str(src / "host_snap.cpp"), str(src / "host_stages.cpp"), str(src / "host_stages_par.cpp"),
           str(src / "gcm_vaes.cpp"),
           str(src / "file_container.cpp"), "-I" + str(ROOT / "include"), "-lcrypto", "-lpthread", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe


def test_host_code_under_tsan(tsan_fuzzer):
    """The same fuzz under ThreadSanitizer: the single-object stage's worker
    pool (ecies_encrypt_par) hands blocks to the calling thread through
    atomics; any race there stops the run."""
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(tsan_fuzzer), "6", "0x5EED"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
