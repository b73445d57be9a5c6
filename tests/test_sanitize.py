"""The host half of the library under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5;
the reference runs its unit tier with `go test -race`, Makefile:284): tests/csrc/sanitize_main.cpp
drives the conjunctive-match compiler, the image builders (IPv4 / IPv6), the delta journal, the
flow-text parser and the Service feature over seeded random rule sets; any sanitizer report aborts
the driver. The HIP entry points (api.cpp) are exercised by the GPU tier."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "antrea_amd", "csrc")
EXE = os.path.join(HERE, "_build", "gpc_sanitize")
SRCS = [os.path.join(HERE, "csrc", "sanitize_main.cpp")] + [os.path.join(CSRC, f) for f in
                                                            ("compiler.cpp", "image.cpp", "flowtext.cpp", "service.cpp")]


@pytest.fixture(scope="module")
def driver():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    deps = SRCS + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hpp")] + \
        [os.path.join(ROOT, "include", "gpc.h")]
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC] + SRCS +
                       ["-o", EXE], check=True)
    return EXE


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_host_library_under_asan_ubsan(driver, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([driver, str(seed), "300"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0 and "sanitize ok" in r.stdout, r.stdout[-4000:]
    assert "runtime error" not in r.stdout and "AddressSanitizer" not in r.stdout, r.stdout[-4000:]
