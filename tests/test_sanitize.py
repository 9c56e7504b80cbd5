"""Host ASan + UBSan run of the C ABI's host code (SURVEY §5 sanitizer
build): `make sanitize` compiles geometry.cpp and every API translation unit
with -fsanitize=address,undefined on the host side only (-Xarch_host; no GPU
sanitizer), links tests/cpp/sanitize_main.cpp, and runs it on the CPU:
geometry planning over a size/parameter sweep plus malformed-argument calls
of every entry point.  Leak checking is off (the HIP runtime keeps its
allocations until exit)."""
import os
import subprocess

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orb-slam-system_amd")


def test_host_code_clean_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-j8", "-C", PKG, "sanitize"], timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([os.path.join(PKG, "build_asan", "sanitize_main")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
