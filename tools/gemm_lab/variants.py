"""Screening-GEMM experiments: source patches of csrc/screen_gemm.hip, built into separate
libraries (_abl/libebert_<name>.so, never shipped) and timed against each other by run.py in
ONE process, interleaved (cdna_hip_programming.md section 5.4 rule 24). A variant that wins is
folded into csrc/screen_gemm.hip by hand; the shipping source carries no ablation switches.

    python tools/gemm_lab/variants.py build [names...]   # on the CPU container
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "robot_ebert_amd", "csrc")
OUT = os.path.join(ROOT, "_abl")

STAGGER = "    if (!(GUARD) && wa) __builtin_amdgcn_s_sleep(1); /* stagger 2nd wave */    \\\n"


def _sub(src, old, new, count=None):
    n = src.count(old)
    if n == 0 or (count is not None and n != count):
        raise SystemExit(f"patch anchor found {n} times: {old[:60]!r}")
    return src.replace(old, new)


def nosleep(src):
    # adopted in csrc/screen_gemm.hip (r2: +2.7 % with hits, +3.7 % without, interleaved)
    return src.replace(STAGGER, "")


def prio_static(src):
    src = nosleep(src)
    return _sub(src, "  int t = 0;\n  // steady state", "  if (wa) __builtin_amdgcn_s_setprio(1);\n"
                "  int t = 0;\n  // steady state", 1)


def prio_static_sleep(src):
    src = _sub(src, "    QP2_ISSUE(4 * t_ + 7", "    if (!(GUARD) && wa) __builtin_amdgcn_s_sleep(1);"
               " \\\n    QP2_ISSUE(4 * t_ + 7", 1)
    return _sub(src, "  int t = 0;\n  // steady state", "  if (wa) __builtin_amdgcn_s_setprio(1);\n"
                "  int t = 0;\n  // steady state", 1)


def grp(n):
    def f(src):
        return _sub(nosleep(src), "constexpr int QP_GROUP_C = 4;", f"constexpr int QP_GROUP_C = {n};", 1)
    return f


def l2only(src):
    # diagnostic: every workgroup reads one of 4 catalog tiles (all catalog fetches hit L2)
    return _sub(src, "const int64_t ct = g * QP_GROUP_C + w % gc;",
                "const int64_t ct = (g * QP_GROUP_C + w % gc) & 3;", 1)


def nobar(src):
    # diagnostic (wrong results): no s_barrier between phases
    return _sub(src, "  asm volatile(\"\" ::: \"memory\");\n  __builtin_amdgcn_s_barrier();\n"
                "  asm volatile(\"\" ::: \"memory\");\n  __builtin_amdgcn_sched_barrier(0);",
                "  asm volatile(\"\" ::: \"memory\");\n"
                "  asm volatile(\"\" ::: \"memory\");\n  __builtin_amdgcn_sched_barrier(0);", 1)


def nowait(src):
    # diagnostic (wrong results): steady-state vmcnt waits dropped
    return _sub(src, "else if constexpr (N == 8) asm volatile(\"s_waitcnt vmcnt(8)\" ::: \"memory\");",
                "else if constexpr (N == 8) asm volatile(\"\" ::: \"memory\");", 1)


def noepi(src):
    # diagnostic: filter epilogue skipped (counts still published)
    return _sub(src, "    if (!cscale && full) filter_tile(std::true_type{});\n"
                "    else filter_tile(std::false_type{});\n", "", 1)


def noepi_nofin(src):
    src = noepi(src)
    return _sub(src, "  if constexpr (FILTER) filter_finish(e, lcnt, q0, QP_TILE, ct);\n}\n", "}\n", 1)


def trivepi(src):
    # diagnostic (wrong results) for the persistent kernel: the epilogue is one sum per lane
    a = src.index("    if constexpr (EPI == EPI_POOL) {\n      pool_quadrant(cur, acc0")
    b = src.index("    // every wave is past its reads of lcnt")
    return src[:a] + """    { float sm = 0.f;
      for (int i = 0; i < 4; ++i) for (int jj = 0; jj < 2; ++jj) for (int r = 0; r < 4; ++r)
        sm += acc0[i][jj][r] + acc1[i][jj][r] + acc2[i][jj][r] + acc3[i][jj][r];
      if (sm == 1234.5f) A->e.ovf[0] = 1; }
""" + src[b:]


def nozero(src):
    # diagnostic (wrong results): the accumulators are not cleared between tiles
    return _sub(src, "      zero_acc();\n      for (int t = 0; t < kt - 2; t += 2) {",
                "      for (int t = 0; t < kt - 2; t += 2) {", 1)


def nocoltest(src):
    # diagnostic (wrong results): the SIMPLE column test is one compare per column on a single
    # accumulator value
    a = src.index("    if constexpr (SIMPLE) {\n#pragma unroll\n      for (int c = 0; c < 4; ++c) {\n        float mx")
    b = src.index("    } else {\n      f32x4_t cs[2][4];")
    return src[:a] + """    if constexpr (SIMPLE) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        colm |= (acc_of(0, c >> 1)[0][c & 1][0] * q4[c] >= t4[c] ? 1u : 0u) << c;
""" + src[b:]


VARIANTS = {"nozero": nozero, "nocoltest": nocoltest, "trivepi": trivepi, "noepi": noepi, "noepi_nofin": noepi_nofin, "l2only": l2only, "nobar": nobar, "nowait": nowait, "grp2": grp(2), "grp8": grp(8), "grp16": grp(16),"base": lambda s: s, "nosleep": nosleep, "prio_static": prio_static,
            "prio_static_sleep": prio_static_sleep}


def build(name):
    ref = os.environ.get("GEMM_LAB_REF")  # e.g. HEAD: patch the committed source instead
    if ":" in name:  # NAME:REF builds variant `base` of commit REF under NAME
        name, ref = name.split(":", 1)
        VARIANTS.setdefault(name, lambda s: s)
    if ref:
        src = subprocess.run(["git", "-C", ROOT, "show", f"{ref}:robot_ebert_amd/csrc/screen_gemm.hip"],
                             check=True, capture_output=True, text=True).stdout
    else:
        src = open(os.path.join(CSRC, "screen_gemm.hip")).read()
    src = VARIANTS[name](src)
    base = os.path.join("/tmp", "gemm_lab", name)
    work = os.path.join(base, "x", "csrc")   # common.h includes ../../include/ebert.h
    os.makedirs(work, exist_ok=True)
    if not os.path.exists(os.path.join(base, "include")):
        os.symlink(os.path.join(ROOT, "include"), os.path.join(base, "include"))
    shutil.copy(os.path.join(CSRC, "common.h"), work)
    with open(os.path.join(work, "screen_gemm.hip"), "w") as f:
        f.write(src)
    obj = os.path.join(work, "screen_gemm.o")
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall",
             "-Wno-unused-function", "-I" + os.path.join(ROOT, "include")]
    subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-c", os.path.join(work, "screen_gemm.hip"),
                                                      "-o", obj], check=True)
    others = [os.path.join(CSRC, "build", f) for f in
              ("api.o", "driver.o", "select_topk.o", "prep.o", "rescore.o", "als.o")]
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, f"libebert_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o", lib, obj]
                   + others + ["-Wl,-rpath,/opt/rocm/lib"], check=True)
    print("built", lib)


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] != "build":
        raise SystemExit(__doc__)
    for n in (sys.argv[2:] or list(VARIANTS)):
        build(n)
