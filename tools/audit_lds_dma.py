"""Wait-state audit of the asm LDS-DMA statements (fm_dma16, csrc/flrelu_mfma.h): compiles the kernels that use it to
gfx950 assembly and, for every `buffer_load_dwordx4 ... lds`, counts the wait states since the last VALU write of an
SGPR the DMA reads (descriptor, soffset: 5 needed) and since the last SALU write of M0 (1 needed).  The compiler pads
these for a builtin but not around an asm statement, so the statement carries its own s_nop; this checks it does.
    python tools/audit_lds_dma.py [-DFBM_OS_DMA=1 ...]     (exit 1 when a DMA is short of wait states)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "image_compression_2_amd", "csrc")
FILES = {"flrelu_mfma.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"], "flrelu_bwd_mfma.hip": []}


def _sgprs(spec):
    m = re.match(r"s\[(\d+):(\d+)\]", spec)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", spec)
    return {int(m.group(1))} if m else set()


def audit(asm_text):
    """-> (number of LDS DMAs, list of (index, what, wait states)) for the DMAs short of wait states (straight-line
    look-back: a branch target in between ends the look-back, which can only make the count conservative)."""
    ins = []
    for line in asm_text.split("\n"):
        t = line.split(";")[0].strip()
        if not t or t.startswith((".", "//")):
            continue
        ins.append(t)
    short, n = [], 0
    for i, t in enumerate(ins):
        if not (t.startswith("buffer_load") and t.endswith(" lds")):
            continue
        n += 1
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        read = _sgprs(ops[1]) | _sgprs(ops[2].split()[0])
        states, need_sg, need_m0 = 0, True, True
        for p in reversed(ins[max(0, i - 12):i]):
            if p.endswith(":"):
                break
            op = p.split()[0]
            dst = p.split(None, 1)[1].split(",")[0].strip() if " " in p else ""
            if need_sg and op.startswith("v_") and _sgprs(dst) & read and states < 5:
                short.append((n, f"VALU write of {dst} read as descriptor/soffset", states))
                need_sg = False
            if need_m0 and op.startswith("s_") and dst == "m0":
                if states < 1:
                    short.append((n, "SALU write of m0", states))
                need_m0 = False
            states += int(p.split()[1]) + 1 if op == "s_nop" else 1
    return n, short


def main():
    extra = sys.argv[1:]
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for f, flags in FILES.items():
            out = os.path.join(tmp, f + ".s")
            cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{os.path.join(ROOT, 'include')}",
                   *flags, *extra, "--cuda-device-only", "-S", os.path.join(CSRC, f), "-o", out]
            subprocess.run(cmd, check=True, capture_output=True)
            n, short = audit(open(out).read())
            print(f"{f} {' '.join(extra)}: {n} LDS DMAs, {len(short)} short of wait states")
            for s in short[:10]:
                print("   ", s)
            bad += len(short)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
