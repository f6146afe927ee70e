"""CPU: the C-ABI library loads and exports every entry point include/hip_serial.h
declares; no compute call is made (there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

from comdb2_amd import hsc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "hip_serial.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*\b((?:hsc|hip)_[a-z_0-9]+)\s*\(", src,
                       flags=re.M)
    return sorted(set(names))


def test_header_lists_match_bindings():
    assert declared_functions() == sorted(hsc.EXPORTS)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(hsc.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "comdb2_amd", "csrc")], check=True)
    lib = hsc.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", hsc.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_struct_layouts_match_header(tmp_path):
    # ctypes mirrors must match the C header (itself a mirror of db/comdb2.h:1105-1124)
    prog = tmp_path / "layout.c"
    prog.write_text("""#include <stdio.h>
#include <stddef.h>
#include "hip_serial.h"
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n",
 sizeof(hsc_currange), offsetof(hsc_currange, islocked), sizeof(hsc_currangearr),
 offsetof(hsc_currangearr, ranges), sizeof(hsc_llog), sizeof(hsc_readsets),
 sizeof(hsc_probe_batch), sizeof(hsc_timing), sizeof(hsc_raw_log),
 offsetof(hsc_raw_log, recon_keys), sizeof(hsc_graph_stats)); return 0;}""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)],
                   check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [ctypes.sizeof(hsc.CurRange), hsc.CurRange.islocked.offset,
            ctypes.sizeof(hsc.CurRangeArr), hsc.CurRangeArr.ranges.offset,
            ctypes.sizeof(hsc._LLog), ctypes.sizeof(hsc._ReadSets),
            ctypes.sizeof(hsc.ProbeBatch), ctypes.sizeof(hsc.Timing), ctypes.sizeof(hsc._RawLog),
            hsc._RawLog.recon_keys.offset, ctypes.sizeof(hsc.GraphStats)]
    assert got == want


def test_no_device_no_context():
    lib = hsc.load()
    if lib.hsc_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(hsc.HscError):
        hsc.Validator(0)
