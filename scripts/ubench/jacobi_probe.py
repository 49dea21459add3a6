"""Probe builds (r05) from a /tmp copy of the sources (the product sources stay unchanged):

  jfixed -- k_epnp5_jacobi_b runs exactly 6 sweeps (no convergence test: every variant runs the
            same step count)
  jcheap -- jfixed, and the rotation parameters from two multiplies instead of jrr_rotation_sel's
            chain (wrong numbers, same data movement): where a latency-form step's time goes
  pack12 -- k_pnp_solve writes 12-double records (R, t; validity left to the status byte) instead
            of 13 doubles at a 16-double stride: its write traffic and time (only that kernel's
            figures mean anything in this build; the records' readers still assume 16)
  novalid -- k_pnp_solve keeps the 16-double stride and leaves the validity slot unwritten: does the
            write traffic follow the written bytes (96 of each 128-byte record) or the lines touched

    python3 scripts/ubench/jacobi_probe.py      -> build/ab/librsac_{jfixed,jcheap,pack12}.so
    then time the kernels under rocprofv3 (scripts/gpu_r05_jprobe.sh)
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXED = [("        if (!(off > 1e-32 * diag)) break;\n        epnp_blk_sweep<0>",
          "        if (sweep >= 6) break;\n        epnp_blk_sweep<0>")]
CHEAP = FIXED + [("    jrr_rotation_sel(sweep, x00, x11, x01, cs, sn);",
                  "    cs = 1.0 - 1e-30 * x00; sn = 1e-30 * x01 * x11;")]


def build(name, edits):
    t = f"/tmp/jprobe_{name}"
    shutil.rmtree(t, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "code-reproduction-ransac_amd", "csrc"), os.path.join(t, "x", "csrc"),
                    ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(t, "include"))
    p = os.path.join(t, "x", "csrc", "rsac_kernels.hip")
    s = open(p).read()
    for old, new in edits:
        if s.count(old) != 1:
            sys.exit(f"anchor not found once: {old[:60]!r}")
        s = s.replace(old, new)
    open(p, "w").write(s)
    out = os.path.join(ROOT, "build", "ab", f"librsac_{name}.so")
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(t, "x", "csrc"), f"OUT={out}"], check=True,
                   stderr=subprocess.DEVNULL)
    print(out)


PACK12 = [("    double *m = a.models + rec * kModelStride;\n    int32_t idx[4];",
           "    double *m = a.models + rec * 12;\n    int32_t idx[4];"),
          ("    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];\n    m[kValidSlot] = st > 0 ? 1.0 : 0.0;\n    a.status[rec] = st;\n"
           "    if (a.counts_out) a.counts_out[rec] = 0;  // the scoring launch",
           "    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];\n    a.status[rec] = st;\n"
           "    if (a.counts_out) a.counts_out[rec] = 0;  // the scoring launch")]

NOVALID = [("    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];\n    m[kValidSlot] = st > 0 ? 1.0 : 0.0;\n    a.status[rec] = st;\n"
            "    if (a.counts_out) a.counts_out[rec] = 0;  // the scoring launch",
            "    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];\n    a.status[rec] = st;\n"
            "    if (a.counts_out) a.counts_out[rec] = 0;  // the scoring launch")]

os.makedirs(os.path.join(ROOT, "build", "ab"), exist_ok=True)
for name in sys.argv[1:] or ["jfixed", "jcheap", "pack12"]:
    build(name, {"jfixed": FIXED, "jcheap": CHEAP, "pack12": PACK12, "novalid": NOVALID}[name])
