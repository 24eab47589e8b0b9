"""ASan + UBSan over the CPU code (the C++ under AddressSanitizer / UndefinedBehaviorSanitizer,
signed-overflow semantics emulated explicitly rather than left as UB): oracle/sanitize_main.cpp drives the
oracle through every operator shape and checks the library's shared host arithmetic (make_div_inv)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_and_host_arithmetic_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "sanitize_main")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "runtime error" not in p.stderr and "ERROR: AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "sanitized run ok" in p.stdout
