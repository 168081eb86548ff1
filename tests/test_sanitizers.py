"""Sanitizer builds: the CPU oracle (oracle/bn_oracle.c) and the
host compilation of the engine's device headers (tests/native/san_emul.cpp),
built with AddressSanitizer + UndefinedBehaviorSanitizer and cross-checked on a
few inputs of each kind by tests/native/san_main.cpp.  Any report fails the
run (-fno-sanitize-recover).  GPU sanitizers are not available on this pool;
the device formulas are covered here through their host compilation.

The instrumented build takes about two minutes; the binary is kept in
tests/native/ (git-ignored) and rebuilt only when a source it depends on changes."""
import glob
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
EXE = os.path.join(NATIVE, "san_main.bin")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-O1"]


def _sources():
    return ([os.path.join(ROOT, "oracle", "bn_oracle.c"), os.path.join(ROOT, "oracle", "bn_oracle.h"),
             os.path.join(NATIVE, "san_emul.cpp"), os.path.join(NATIVE, "san_main.cpp")]
            + glob.glob(os.path.join(ROOT, "paritytech-bn_amd", "csrc", "*.h"))
            + [os.path.join(ROOT, "paritytech-bn_amd", "csrc", "constants.inc")])


def _build():
    if os.path.exists(EXE) and os.path.getmtime(EXE) >= max(os.path.getmtime(s) for s in _sources()):
        return
    o1, o2 = EXE + ".oracle.o", EXE + ".emul.o"
    jobs = [["gcc", "-std=gnu11", "-fno-strict-aliasing", "-c", "-o", o1,
             os.path.join(ROOT, "oracle", "bn_oracle.c")] + SAN,
            ["g++", "-std=c++17", "-DBN_HOST_CHECKS", "-c", "-o", o2, os.path.join(NATIVE, "san_emul.cpp")] + SAN]
    with ThreadPoolExecutor(2) as ex:
        for f in [ex.submit(subprocess.check_call, j) for j in jobs]:
            f.result()
    subprocess.check_call(["g++", "-std=c++17", "-o", EXE, os.path.join(NATIVE, "san_main.cpp"), o1, o2,
                           "-lpthread"] + SAN)
    for o in (o1, o2):
        os.remove(o)


@pytest.mark.timeout(900)
@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_asan_ubsan_oracle_and_device_formulas():
    _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([EXE], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "san ok" in r.stdout
