"""Host code under ASan + UBSan (SURVEY.md §5 race detection / sanitizers):
the library rebuilt with every host function instrumented (`make asan`:
comdb2_amd/lib/san/libhsc_san.so; device code untouched) runs the host-only
tests that drive the untrusted-bytes decoders (raw log records, OSQL_SERIAL
payloads, their fuzzed mutations), the marshaller, the incremental log
decode and the CurRangeArr harness, in a python subprocess with the clang
ASan runtime preloaded.  Any sanitizer report fails the run
(halt_on_error)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_LIB = os.path.join(ROOT, "comdb2_amd", "lib", "san", "libhsc_san.so")
HOST_TESTS = ["tests/test_decoder_fuzz.py", "tests/test_logdec.py", "tests/test_wire.py",
              "tests/test_marshal.py", "tests/test_incremental.py", "tests/test_abi.py",
              "tests/test_coalesce.py", "tests/test_recon.py"]


def asan_runtime():
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-print-file-name=libclang_rt.asan-x86_64.so"],
                       capture_output=True, text=True)
    path = r.stdout.strip()
    return path if r.returncode == 0 and os.path.isabs(path) and os.path.exists(path) else None


def test_host_code_under_asan_ubsan():
    rt = asan_runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "comdb2_amd", "csrc"), "asan"],
                   check=True)
    syms = subprocess.run(["nm", "-D", SAN_LIB], capture_output=True,
                          text=True).stdout
    assert "__asan_" in syms and "__ubsan_" in syms  # really instrumented
    env = dict(os.environ)
    pre = env.get("LD_PRELOAD", "")
    env["LD_PRELOAD"] = rt + (":" + pre if pre else "")
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["HSC_LIB"] = SAN_LIB
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu",
                        "-p", "no:cacheprovider", *HOST_TESTS], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=1200)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error" not in tail, tail
