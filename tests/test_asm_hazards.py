"""Static check of the MFMA data hazards in the kernels that issue MFMAs from inline asm (CPU test).

hipcc inserts the wait states an MFMA's results and operands need only for the builtins; for an
`asm volatile("v_mfma ...")` it sees an opaque statement.  The d-256 attention forward issues its P.V MFMAs
from asm (flash.hip, attn_fwd256w_kernel), the persistent GEMMs all of theirs (gemm_w4.hip).  This test
compiles those files to gfx950 assembly and scans every kernel's straight-line code for the hazards hipcc
cannot have resolved, i.e. those with an inline-asm instruction (between ;;#ASMSTART / ;;#ASMEND) on either
side:
  * an instruction touching registers an asm MFMA writes before that MFMA's result is ready (18 wait states
    after a 32x32x16, 10 after a 16x16x32; MFMAs accumulating into the same registers are exempt: back-to-back
    accumulation is interlocked), or an asm instruction reading a builtin MFMA's result that early, and
  * an asm MFMA reading a register a VALU instruction wrote less than 2 wait states earlier.
Wait states are counted as 1 per instruction and N + 1 per `s_nop N` (conservative: an MFMA issue takes
more).  Branch targets reset the window.  Hazards between two compiler-built instructions are hipcc's to
resolve (its hazard recognizer knows the exact rules) and are not checked.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "projectiontrainer_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        f = m.group(1)
        if m.group(4) is not None:
            out.add((f, int(m.group(4))))
        else:
            out.update((f, i) for i in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(line):
    """(mnemonic, dst regs, src regs) of one instruction line, or None."""
    line = line.split(";")[0].split("//")[0].strip()
    if not line or line.endswith(":") or line.startswith("."):
        return None
    parts = line.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    if op.startswith(("s_", "buffer_store", "global_store", "scratch_store", "ds_write")) or not ops:
        return op, set(), regs(" ".join(ops))
    return op, regs(ops[0]), regs(" ".join(ops[1:]))


def kernels(asm):
    cur, body = None, []
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            if "s_endpgm" in line:
                yield cur, body
                cur, body = None, []
            else:
                body.append(line)


def hazards(body):
    found = []
    pending = []   # (regs, wait states left, index, from asm)
    valu_recent = []   # (regs, wait states left, index)
    in_asm = False
    for i, line in enumerate(body):
        t = line.strip()
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if re.match(r"^\.LBB\S*:", t):
            pending, valu_recent = [], []
            continue
        p = parse(line)
        if p is None:
            continue
        op, dst, src = p
        ws = int(re.search(r"s_nop\s+(\d+)", line).group(1)) + 1 if op == "s_nop" else 1
        is_mfma = op.startswith("v_mfma")
        if is_mfma:
            srcs = [regs(x) for x in line.split(";")[0].split(None, 1)[1].split(",")[1:]]
            a_b = srcs[0] | srcs[1] if len(srcs) >= 2 else set()
            c = srcs[2] if len(srcs) >= 3 else set()
            for r, left, j, asm in pending:
                if not (asm or in_asm):
                    continue
                if r & a_b:
                    found.append((j, i, "MFMA result read as A/B too early"))
                if r & c and r != dst:
                    found.append((j, i, "MFMA result read as C by a different accumulation"))
            if in_asm:
                for r, left, j in valu_recent:
                    if r & (a_b | c):
                        found.append((j, i, "VALU write read by an asm MFMA without 2 wait states"))
        elif op not in ("s_nop", "s_waitcnt") and not op.startswith("s_"):
            for r, left, j, asm in pending:
                if (asm or in_asm) and r & (src | dst):
                    found.append((j, i, f"MFMA result touched by {op} before it is ready"))
        # age the windows
        pending = [(r, left - ws, j, a) for r, left, j, a in pending if left - ws > 0]
        valu_recent = [(r, left - ws, j) for r, left, j in valu_recent if left - ws > 0]
        if is_mfma:
            need = 18 if "32x32" in op else 10
            pending = [(r, left, j, a) for r, left, j, a in pending if not (r & dst)]
            pending.append((dst, need, i, in_asm))
        elif op.startswith("v_") and dst:
            valu_recent.append((dst, 2, i))
    return found


@pytest.mark.parametrize("src", ["flash.hip", "gemm_w4.hip"])
def test_inline_asm_mfma_hazards(src, tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path / (src + ".s")
    subprocess.check_call([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                           "-I", CSRC, os.path.join(CSRC, src), "-o", str(out)],
                          stderr=subprocess.DEVNULL)
    asm = out.read_text()
    bad = []
    for name, body in kernels(asm):
        for j, i, what in hazards(body):
            bad.append(f"{name}: {what}: [{j}] {body[j].strip()} -> [{i}] {body[i].strip()}")
    assert not bad, "\n".join(bad[:20])


def test_hazard_scanner_catches_known_patterns():
    """The scanner itself: the two hazards it exists for are flagged, a padded sequence is not."""
    A, E = ";;#ASMSTART", ";;#ASMEND"
    read_early = [A, "v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], 0", E, "v_max3_f32 v30, v0, v1, v2"]
    assert hazards(read_early)
    asm_reads_builtin = ["v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], 0", A, "v_max3_f32 v30, v0, v1, v2", E]
    assert hazards(asm_reads_builtin)
    copy_then_mfma = ["v_accvgpr_write_b32 a0, v5", A, "v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], a[0:3], v[0:15]", E]
    assert hazards(copy_then_mfma)
    compiler_only = ["v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], 0", "v_max3_f32 v30, v0, v1, v2"]
    assert not hazards(compiler_only)
    padded = [A, "v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], 0", E, "s_nop 7", "s_nop 7", "s_nop 3",
              "v_max3_f32 v30, v0, v1, v2", "v_cvt_pk_bf16_f32 v40, v30, v31",
              A, "s_nop 2", "v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[40:43], v[0:15]", E,
              A, "v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]", E]
    assert not hazards(padded)
