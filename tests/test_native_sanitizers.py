"""Race detection / sanitizers for the native host runtime.

``tests/native/loader_stress.cpp`` drives the C++ token loader (producer threads, the
consumer, concurrent random-access fills, seeks, close with blocked producers) and is
built twice here: with ThreadSanitizer and with AddressSanitizer + UBSan.  Host code
only -- the loader has no HIP dependency.  The TSan build found a real race (the epoch
permutation cache, fixed in ``runtime/csrc/loader.cpp``)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "loader_stress.cpp")

FLAVOURS = {
    "tsan": ["-fsanitize=thread"],
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
}


@pytest.mark.parametrize("flavour", sorted(FLAVOURS))
def test_loader_under_sanitizer(flavour, tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / f"loader_stress_{flavour}")
    build = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-pthread", *FLAVOURS[flavour], SRC, "-o", exe],
                           capture_output=True, text=True, timeout=300)
    if build.returncode != 0 and "cannot find" in build.stderr:
        pytest.skip(f"{flavour} runtime not installed: {build.stderr[-300:]}")
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, TMPDIR=str(tmp_path), TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert run.returncode == 0 and "loader stress OK" in run.stdout, (run.stdout[-2000:], run.stderr[-6000:])
