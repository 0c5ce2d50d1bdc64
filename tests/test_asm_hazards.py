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


# every HIP source of libptk.so (capi / models / comm are host code)
PRODUCT_SOURCES = ["flash.hip", "gemm_w4.hip", "gemm_tn.hip", "gemm.hip", "norm.hip", "attn.hip", "misc.hip", "image.hip",
                   "train.hip"]
_ASM_CACHE = {}


def product_asm(src, tmp_dir):
    """gfx950 assembly of one product source; the first call compiles every product source in parallel."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    if not _ASM_CACHE:
        from concurrent.futures import ThreadPoolExecutor

        def build(f):
            out = os.path.join(str(tmp_dir), f + ".s")
            subprocess.check_call([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                                   "-S", "-I", CSRC, os.path.join(CSRC, f), "-o", out], stderr=subprocess.DEVNULL)
            return f, open(out).read()
        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            _ASM_CACHE.update(ex.map(build, PRODUCT_SOURCES))
    return _ASM_CACHE[src]


@pytest.fixture(scope="module")
def asm_dir(tmp_path_factory):
    return tmp_path_factory.mktemp("asm")


@pytest.mark.parametrize("src", ["flash.hip", "gemm_w4.hip", "gemm_tn.hip"])
def test_inline_asm_mfma_hazards(src, asm_dir):
    asm = product_asm(src, asm_dir)
    bad = []
    for name, body in kernels(asm):
        for j, i, what in hazards(body):
            bad.append(f"{name}: {what}: [{j}] {body[j].strip()} -> [{i}] {body[i].strip()}")
    assert not bad, "\n".join(bad[:20])


# ---- register spills.  The round-3 split-tail GEMM (commit 982c7a5, reverted in 44564ce) pushed
# gemm_p8_kernel to 81 SGPR spills; under that pressure hipcc moved the 128 MFMA accumulators of
# gemm_p8_kernel<ACT_GELU_ERF_BWD> between AGPRs and VGPRs right after the inline-asm MFMAs that wrote them
# (v_accvgpr_read 0 wait states after the MFMA: 372 hazards by the scanner above, which did not exist yet),
# so the projector backward summed garbage whether or not the split ran.  Spill counts are therefore pinned
# per kernel: SGPR spills go to VGPR lanes (v_writelane / v_readlane, no memory traffic), the only VGPR spills
# (scratch) are the d-256 dK/dV kernels' epilogue stores of 16 accumulators; a kernel whose counts grow, a new
# kernel that spills, or a scratch access inside a loop fails.
SPILL_BUDGET = {   # kernel symbol substring -> (sgpr_spill_count, vgpr_spill_count, private_segment bytes)
    "attn_bwd_dkv256b_kernel": (27, 16, 68),
    "attn_dkv_reduce_kernel": (19, 0, 0),
    # the persistent d-256 forward: the per-item state and arguments live across the item loop; every spill
    # reload sits in the per-item code (the K / V tile loop has none: v_readlane count 0 there, r05)
    "attn_fwd256w_kernel": (52, 0, 0),
    "attn_bwd_dq256w_kernel": (38, 0, 0),   # the persistent dQ's per-item state (r05; none in the K/V tile loop)
    "attn_bwd_dkv256_kernelILi32E": (15, 13, 56),
    # the persistent kernels' epilogues read their arguments through a laundered kernarg pointer
    # (gemm_w4.hip kernarg_args, scalar loads): 0 spills, except the GELU-erf epilogues (the projector's) and
    # the stream-K tail variants' bookkeeping (r05: 24 -> 0-1 with the in-kernel reducer moved to p8_fixup_kernel)
    "gemm_p8_kernelILi0ELi0ELb1E": (1, 0, 0),
    "gemm_tn_kernelILi0ELb1E": (3, 0, 0),
    "Lb0ELi224E": (1, 0, 0),   # the 8-wave kernel's 224- / 192-row tiles, general epilogues
    "Lb0ELi192E": (1, 0, 0),
    "Lb0ELi160E": (3, 0, 0),   # (the general GELU-tanh epilogue of the 160-row tiles: 3)
    "gemm_p8_kernelILi1ELi0ELb0E": (4, 0, 0),
    # GELU-erf epilogues: 28 / 20 -> 31 / 28 with the K-slice (zslices) DMA offsets (r05); none in the K loop
    "gemm_p8_kernelILi2ELi0ELb0E": (31, 0, 0),
    "gemm_p8_kernelILi4ELi0ELb0E": (28, 0, 0),
    # the 4-wave kernel's GELU-erf epilogues (not dispatched: the projector's GELU-erf shapes run on p8), with the
    # whole-line stores' row-pair exchange
    "gemm_w4_kernelILi2ELi0E": (18, 0, 0),
    "gemm_w4_kernelILi4ELi0E": (14, 0, 0),
    "gemm_big2_kernelILi0ELi0E": (28, 0, 0),   # + the stats_only early-out of the row-statistics epilogue
    "gemm_big2_kernelILi1ELi0E": (11, 0, 0),
    "gemm_big2_kernelILi2ELi0E": (25, 0, 0),
    "gemm_big2_kernelILi4ELi0E": (11, 0, 0),
    "gemm_big_kernelILi0ELi0E": (28, 0, 0),
    "gemm_big_kernelILi1ELi0E": (11, 0, 0),
    "gemm_big_kernelILi2ELi0E": (25, 0, 0),
    "gemm_big_kernelILi4ELi0E": (11, 0, 0),
    "gemm_nt_kernelILi2ELi0E": (5, 0, 0),
    "gemm_nt_kernelILi4ELi0E": (1, 0, 0),
    "qknorm_rope_bwd_kernelILi4E": (28, 0, 0),
}


def kernel_resources(asm):
    """{kernel symbol: (sgpr_spill_count, vgpr_spill_count, private_segment_fixed_size)} from the amdhsa
    metadata of one assembly file."""
    md = asm[asm.find("amdhsa.kernels:"):]
    out = {}
    for ent in re.split(r"\n  - ", md)[1:]:
        m = re.search(r"\.name:\s+(\S+)", ent)
        if not m:
            continue

        def g(k):
            v = re.search(r"\.%s:\s+(\d+)" % k, ent)
            return int(v.group(1)) if v else 0
        out[m.group(1)] = (g("sgpr_spill_count"), g("vgpr_spill_count"), g("private_segment_fixed_size"))
    return out


def loop_scratch(body):
    """Scratch spill / reload instructions inside a loop (hipcc tags loop blocks `; in Loop:` / `Loop Header`)."""
    bad, in_loop = [], False
    for line in body:
        t = line.strip()
        if re.match(r"^\.LBB\S*:", t):
            in_loop = "Loop" in t
            continue
        if in_loop and re.match(r"^(scratch_|buffer_(store|load)\S*\s.*\boff(set)?\b.*s\[0:3\])", t):
            bad.append(t)
    return bad


@pytest.mark.parametrize("src", PRODUCT_SOURCES)
def test_kernel_spills_within_budget(src, asm_dir):
    asm = product_asm(src, asm_dir)
    res = kernel_resources(asm)
    assert res, "no kernel metadata parsed"
    bad = []
    for name, got in res.items():
        budget = next((b for k, b in SPILL_BUDGET.items() if k in name), (0, 0, 0))
        if any(x > y for x, y in zip(got, budget)):
            bad.append(f"{name}: (sgpr spills, vgpr spills, private bytes) = {got} > budget {budget}")
    for name, body in kernels(asm):
        for t in loop_scratch(body):
            bad.append(f"{name}: scratch access inside a loop: {t}")
    assert not bad, "\n".join(bad[:20])


@pytest.mark.parametrize("src", ["flash.hip", "gemm_w4.hip", "gemm_tn.hip"])
def test_asm_never_writes_m0(src, asm_dir):
    """LDS-DMA asm takes its LDS address through the {m0} constraint (hipcc writes M0 and knows the asm reads
    it); an M0 write hidden inside an asm statement would break any M0 value hipcc keeps live."""
    asm = product_asm(src, asm_dir)
    bad = []
    for name, body in kernels(asm):
        in_asm = False
        for line in body:
            t = line.strip()
            if t.startswith(";;#ASMSTART"):
                in_asm = True
            elif t.startswith(";;#ASMEND"):
                in_asm = False
            elif in_asm:
                p = parse(line)
                if p and p[0].startswith("s_") and re.match(r"^\S+\s+m0\b", t):
                    bad.append(f"{name}: {t}")
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
    # the spill checks
    loop_body = [".LBB3_9:                                ; =>This Inner Loop Header: Depth=1",
                 "scratch_store_dwordx4 off, a[0:3], off  ; 16-byte Folded Spill", ".LBB3_41:",
                 "scratch_load_dwordx4 v[12:15], off, off offset:48 ; 16-byte Folded Reload"]
    assert loop_scratch(loop_body) == ["scratch_store_dwordx4 off, a[0:3], off  ; 16-byte Folded Spill"]
    md = "amdhsa.kernels:\n  - .name: k\n    .sgpr_spill_count: 3\n    .vgpr_spill_count: 0\n"
    assert kernel_resources(md) == {"k": (3, 0, 0)}
