"""The ctypes mirrors in gwa.py have the layout of the C structs in include/gwa.h.

A C program generated from the ctypes field lists prints sizeof() and offsetof() of every field of
the corresponding C struct (a field name missing on the C side fails its compilation); the test
compares them with ctypes.  This is what keeps the host-side mirror of the boundary honest when a
field is appended on one side only.  CPU only: gcc and the header, no GPU, no library calls.
"""
import json
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "genome-weaver-align_amd"))

import gwa  # noqa: E402  (the module loads; nothing here calls into libgwa)

PAIRS = [
    ("gwa_config_t", gwa._Config),
    ("gwa_reads_t", gwa._Reads),
    ("gwa_read_buf_t", gwa._ReadBuf),
    ("gwa_record_t", gwa.Record),
    ("gwa_results_t", gwa._Results),
    ("gwa_batch_stats_t", gwa.BatchStats),
    ("gwa_pipeline_stats_t", gwa.PipelineStats),
]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_ctypes_mirrors_match_c_layout(tmp_path):
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "gwa.h"', "int main(void) {", 'printf("{");']
    first = True
    for cname, cls in PAIRS:
        for f in [("__size__", None)] + [(n, t) for n, t in cls._fields_]:
            name = f[0]
            expr = "sizeof(%s)" % cname if name == "__size__" else "offsetof(%s, %s)" % (cname, name)
            sep = "" if first else ","
            first = False
            lines.append('printf("%s\\"%s.%s\\": %%zu", (size_t)%s);' % (sep, cname, name, expr))
    lines += ['printf("}\\n");', "return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    c = json.loads(subprocess.check_output([str(exe)]).decode())
    for cname, cls in PAIRS:
        assert c["%s.__size__" % cname] == __import__("ctypes").sizeof(cls), cname
        for n, _ in cls._fields_:
            assert c["%s.%s" % (cname, n)] == getattr(cls, n).offset, "%s.%s" % (cname, n)
