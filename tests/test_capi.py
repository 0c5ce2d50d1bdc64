"""C-ABI checks that need no GPU: libptk.so loads, exports every function
include/ptk.h declares, and the ctypes mirrors of the public structs have the
same size and field offsets as the C compiler gives them (gcc on ptk.h)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ptk.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ptk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from projectiontrainer_amd import _lib as L
    lib = L.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
        assert n in L.SIGNATURES, f"{n} missing from the ctypes binding"
    assert lib.ptk_abi_version() == L.ABI_VERSION == 8


def test_error_reporting_without_gpu():
    """Argument validation runs before any device call."""
    from projectiontrainer_amd import _lib as L
    d = L.GemmDesc()
    d.M, d.N, d.K, d.lda, d.ldb = 64, 64, 60, 64, 64
    d.batch = 1
    rc = L.lib().ptk_gemm(d, None)
    assert rc != 0 and b"multiple of 64" in L.lib().ptk_last_error()


STRUCTS = {
    "ptk_rowmap": ("RowMap", ["g", "skip", "gs", "off"]),
    "ptk_gemm_desc": ("GemmDesc", None),
    "ptk_flash_desc": ("FlashDesc", None),
    "ptk_flash_bwd_desc": ("FlashBwdDesc", None),
    "ptk_siglip_config": ("SiglipConfigC", None),
    "ptk_siglip_layer": ("SiglipLayerC", None),
    "ptk_siglip_weights": ("SiglipWeightsC", None),
    "ptk_projector": ("ProjectorC", None),
    "ptk_gemma3_config": ("Gemma3ConfigC", None),
    "ptk_gemma3_layer": ("Gemma3LayerC", None),
    "ptk_gemma3_weights": ("Gemma3WeightsC", None),
    "ptk_gemma3_batch": ("Gemma3BatchC", None),
    "ptk_gemma3_layer_grads": ("Gemma3LayerGradsC", None),
    "ptk_gemma3_grads": ("Gemma3GradsC", None),
    "ptk_image_desc": ("ImageDesc", None),
    "ptk_gemma3_generate_desc": ("Gemma3GenerateC", None),
    "ptk_gemma3_decode_desc": ("Gemma3DecodeC", None),
}


def test_struct_layouts_match_c_compiler():
    from projectiontrainer_amd import _lib as L
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, (pyname, _) in STRUCTS.items():
        cls = getattr(L, pyname)
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _t in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "t.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(td, "t")
        subprocess.check_call(["gcc", "-o", exe, c])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = {}
    for ln in out:
        if ln:
            a, b, v = ln.split()
            got[(a, b)] = int(v)
    for cname, (pyname, _) in STRUCTS.items():
        cls = getattr(L, pyname)
        assert ctypes.sizeof(cls) == got[(cname, "sizeof")], cname
        for fname, _t in cls._fields_:
            assert getattr(cls, fname).offset == got[(cname, fname)], (cname, fname)
