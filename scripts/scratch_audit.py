"""Where the kernels touch scratch ("0 B/lane scratch on the item path").

Compiles md_kernels.hip to gfx950 assembly (device only, the Makefile's flags) and counts the
scratch loads / stores of every function.  For md_wq_kernel it also reports where they sit: the
kernel's own scratch accesses all come before its first workgroup barrier (the kernel prologue,
the weight image's first load), so the item loop -- wq_tile and wq_vn inlined -- executes
none; the frame the resource report shows (ScratchSize) belongs to the noinline group-section
callees (wq_group, wq_env and the environment step under them).
  python scripts/scratch_audit.py [out.txt]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mdcommunity_amd", "csrc")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        subprocess.run([CLANG, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-I../../include",
                        "-x", "hip", "--cuda-device-only", "-S", "md_kernels.hip", "-o", asm], cwd=CSRC, check=True)
        lines = open(asm).read().splitlines()
    funcs, cur = {}, None
    for ln in lines:
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", ln)
        if m and not m.group(1).startswith("."):
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None:
            funcs[cur].append(ln)
    rep = ["scratch instructions per device function (stores, loads); functions with none omitted:"]
    for f, body in funcs.items():
        st = sum("scratch_store" in x for x in body)
        ld = sum("scratch_load" in x for x in body)
        if st or ld:
            rep.append("  %4d %4d  %s" % (st, ld, f))
    wq = funcs.get("_ZN2md12md_wq_kernelENS_6ParamsEPKf", [])
    ins = [x for x in wq if x.startswith("\t") and not x.strip().startswith(";") and not x.strip().startswith(".")]
    first_bar = next((i for i, x in enumerate(ins) if "s_barrier" in x), len(ins))
    scr = [i for i, x in enumerate(ins) if "scratch_" in x]
    calls = sum("s_swappc" in x for x in ins)
    rep.append("md_wq_kernel: %d instructions, first s_barrier at instruction %d; scratch accesses at %s; "
               "%d calls (the noinline group-section and wait functions)" % (len(ins), first_bar, scr, calls))
    rep.append("item loop (everything after the prologue's barrier): %d scratch instructions"
               % sum(1 for i in scr if i > first_bar))
    txt = "\n".join(rep)
    print(txt)
    if out:
        with open(out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
