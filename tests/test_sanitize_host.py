"""CPU: the host planning arithmetic of libebert under AddressSanitizer + UndefinedBehavior-
Sanitizer (sanitizer build of the host layer).

`make -C robot_ebert_amd/csrc sanitize` builds tests/sanitize/plan_fuzz.hip -- which includes
api.hip (the workspace layouts ws_layout / spec_params, the plan queries) and links the other
sources' host code -- with -fsanitize=address,undefined on the host side only (no GPU
sanitizer exists on this pool), then the binary walks ~45K layouts: batch sizes 1-16384,
catalogs 1-50M rows, k' 4-4096, chunk sizes and flags, plus the self-contained path's sizing
(ebt_catalog_state_bytes, ebt_workspace_bytes). Any sanitizer report aborts it
(-fno-sanitize-recover); its own checks: regions inside the byte count, 256-byte aligned and
ordered, plan == layout. No GPU call is made.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "robot_ebert_amd", "csrc")


def test_planning_arithmetic_under_asan_ubsan():
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", CSRC, "sanitize", f"-j{jobs}"], check=True, timeout=900,
                   stdout=subprocess.DEVNULL)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    out = subprocess.run([os.path.join(CSRC, "build_san", "plan_fuzz")], capture_output=True,
                         text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr
    assert " 0 failures" in out.stdout, out.stdout
