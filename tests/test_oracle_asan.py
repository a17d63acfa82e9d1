"""CPU: the oracle (the parity checker) under AddressSanitizer + UBSan (host
code only).  `make -C oracle asan` builds oracle/asan_driver.cpp with qie_oracle.cpp; the
driver runs prompt forwards, decode steps to the last KV-cache row, attention, sampling
and RoPE tables on odd-sized tiny models in all three summation orders."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "asan_driver")], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0 and "asan ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
