"""The drop-in boundary on the CPU tier: the product library loads, exports every entry point the
public headers declare, and its record layouts match the host-side dtypes. No compute call is made
without a GPU; creating an engine on a machine without one must fail loudly (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from fluidframework_amd import native
from fluidframework_amd import oplog as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("mt_engine.h", "mt_oplog.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(mt_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_the_engine_api():
    names = declared_functions()
    for n in ("mt_engine_create", "mt_engine_submit", "mt_engine_run", "mt_engine_sync", "mt_engine_digests",
              "mt_engine_get_length", "mt_engine_get_text", "mt_engine_dump", "mt_engine_errors"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(native.lib_path("libmtreplay.so"))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_product_library_does_not_contain_the_oracle():
    out = subprocess.run(["nm", "-D", "--defined-only", native.lib_path("libmtreplay.so")], capture_output=True,
                         text=True, check=True).stdout
    assert "mto_" not in out
    assert "mt_engine_run" in out


def test_record_layouts_match_host_dtypes(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text("""
#include <stddef.h>
#include <stdio.h>
#include "mt_oplog.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(mt_op_rec), offsetof(mt_op_rec, seq),
         offsetof(mt_op_rec, pos1), offsetof(mt_op_rec, text_off), offsetof(mt_op_rec, props),
         sizeof(mt_props_rec), sizeof(mt_kv), offsetof(mt_kv, value));
  return 0;
}
""")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    d = ol.OP_DTYPE
    assert got == [d.itemsize, d.fields["seq"][1], d.fields["pos1"][1], d.fields["text_off"][1],
                   d.fields["props"][1], ol.PROPS_DTYPE.itemsize, ol.KV_DTYPE.itemsize, ol.KV_DTYPE.fields["value"][1]]


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU failure mode")
def test_engine_fails_loudly_without_a_gpu():
    from fluidframework_amd.engine import Engine, EngineError
    with pytest.raises(EngineError):
        Engine(1)
