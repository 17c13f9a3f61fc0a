"""CPU checks of the drop-in boundary: libaz loads and exports every symbol
include/*.h declares (az.h, az_chess.h); the ctypes structs match the header layout."""
import ctypes
import os
import re

import numpy as np
import pytest

from custom_alphazero import engine as az

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    names = set()
    for h in sorted(os.listdir(os.path.join(REPO, "include"))):
        if h.endswith(".h"):
            src = open(os.path.join(REPO, "include", h)).read()
            names |= set(re.findall(r"^(?:int|const char\*)\s+(az_\w+)\(", src, re.M))
    return sorted(names)


def test_header_and_binding_agree():
    declared = header_functions()
    assert declared == sorted(az.EXPORTED)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(az.LIB_PATH):
        pytest.fail("libaz.so missing: run __graft_entry__.build()")
    lib = ctypes.CDLL(az.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name
    L = az.load_library()
    assert L.az_abi_version() == 10


def test_product_library_is_not_a_diagnostic_build():
    """The shipped libaz.so carries no diagnostic compile flags (EXTRA= in
    csrc/Makefile: phase stamps, A/B knobs), and its build id is the hash of
    the sources in this tree (what profiles/ record, bench.py matches)."""
    import hashlib
    ident, flags = az.build_id()
    assert flags == "", flags
    csrc = os.path.join(REPO, "custom-alphazero_amd", "csrc")
    names = sorted(f for f in os.listdir(csrc) if f.startswith("az_") and f.endswith((".hip", ".h")))
    paths = [os.path.join(csrc, f) for f in names] + [os.path.join(REPO, "include", "az.h"),
                                                      os.path.join(REPO, "include", "az_chess.h"),
                                                      os.path.join(csrc, "Makefile")]
    h = hashlib.sha256(b"".join(open(p, "rb").read() for p in paths)).hexdigest()[:16]
    assert ident == h, (ident, h)


def _header_structs():
    """{struct name: [field names]} of every `typedef struct x { ... } x;` in include/*.h"""
    out = {}
    for h in sorted(os.listdir(os.path.join(REPO, "include"))):
        if not h.endswith(".h"):
            continue
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", h)).read(), flags=re.S)
        for name, body in re.findall(r"typedef struct (\w+) \{(.*?)\} \1;", src, re.S):
            fields = []
            for decl in body.split(";"):
                decl = decl.strip()
                if not decl:
                    continue
                # "int32_t filters, depth, value_hidden" or "uint64_t pieces[6]"
                _, rest = decl.split(None, 1) if not decl.startswith("const ") else decl[6:].split(None, 1)
                for v in rest.split(","):
                    fields.append(re.sub(r"\[.*\]", "", v).strip().lstrip("*"))
            out[name] = fields
    return out


def _compiler_layout(structs):
    """sizeof and offsetof of every field, printed by a C program built from the headers with gcc."""
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "az.h"', '#include "az_chess.h"',
             "int main(void) {"]
    for name, fields in structs.items():
        lines.append(f'  printf("{name} sizeof %zu\\n", sizeof({name}));')
        for f in fields:
            lines.append(f'  printf("{name} {f} %zu\\n", offsetof({name}, {f}));')
    lines += ["  return 0;", "}"]
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "probe.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "probe")
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        text = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    lay = {}
    for ln in text.splitlines():
        s_, f, v = ln.split()
        lay.setdefault(s_, {})[f] = int(v)
    return lay


def test_struct_layouts_match_the_compiler():
    """Every header struct's size and every field's offset, as gcc lays out
    include/*.h, equal the ctypes / numpy bindings' (a reordered field of the
    same total size fails here)."""
    structs = _header_structs()
    assert set(structs) == {"az_config", "az_tensor", "az_stats", "az_chess_pos", "az_chess_config"}
    lay = _compiler_layout(structs)
    from custom_alphazero.chess import kernels as K
    bindings = {"az_config": az.Config, "az_tensor": az.Tensor, "az_stats": az.Stats,
                "az_chess_config": az.ChessConfig}
    for name, cls in bindings.items():
        assert lay[name]["sizeof"] == ctypes.sizeof(cls), name
        assert [f for f, _ in cls._fields_] == structs[name], name
        for f, _ in cls._fields_:
            assert getattr(cls, f).offset == lay[name][f], (name, f)
    assert lay["az_chess_pos"]["sizeof"] == K.POS_DTYPE.itemsize
    assert list(K.POS_DTYPE.names) == structs["az_chess_pos"]
    for f in K.POS_DTYPE.names:
        assert K.POS_DTYPE.fields[f][1] == lay["az_chess_pos"][f], f


def test_engine_fails_loudly_without_gpu():
    """No CPU fallback: without a visible HIP device the engine refuses to
    start (the product path never routes through the oracle)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from custom_alphazero import engine as az
    with pytest.raises(az.AzError, match="no HIP device"):
        az.Engine(6, 7, 4, True, 10, slots=4, evaluator=az.EVAL_SYNTHETIC)


def test_chess_kernels_fail_loudly_without_gpu():
    """The chess board seam has no CPU fallback either."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from custom_alphazero.chess import kernels as K
    from custom_alphazero.chess.board import Board
    b = Board()  # construction is host bookkeeping only
    with pytest.raises(az.AzError, match="no HIP device"):
        b.moves
    with pytest.raises(az.AzError, match="no HIP device"):
        K.encode(np.zeros((1, 8), K.POS_DTYPE), np.ones((1, 8), np.uint8))


def test_integration_stub_matches_the_header():
    """INTEGRATION.md's ctypes stub (what a maintainer would paste into the
    reference) declares az_config and az_tensor field for field as
    include/az.h does."""
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    hdr = _header_structs()
    for name in ("az_config", "az_tensor"):
        m = re.search(r"class %s\(ctypes\.Structure\):\s*_fields_ = \[(.*?)\]\n" % name, doc, re.S)
        assert m, name
        fields = re.findall(r'\("(\w+)"', m.group(1))
        assert fields == hdr[name], (name, fields, hdr[name])
