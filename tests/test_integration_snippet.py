"""CPU: the reference-side bindings shown in INTEGRATION.md (section 2: the aggregator; section 5: the
compute node's per-client states) compile.

The block is extracted verbatim from INTEGRATION.md and compiled (syntax and types, -fsyntax-only)
against the reference's own headers (/root/reference/pipeline_simulation/systemAPI.h, Task.h, State.h,
network_layer.h; models/), libtorch's headers and include/fedavg/fa.h -- so the documented drop-in for
aggregator.cpp:55-167 is known to build.  Needs the reference tree (build container only).
"""
import os
import re
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"


def snippet(name="aggregator_fa"):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```cpp\n(// %s\.cpp.*?)```" % re.escape(name), text, re.S)
    assert m, "INTEGRATION.md binding block %s not found" % name
    return m.group(1)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "pipeline_simulation")), reason="needs /root/reference")
@pytest.mark.parametrize("name,syms", [
    ("aggregator_fa", ("fa_create", "fa_bucket_define", "fa_submit", "fa_finalize", "fa_reduce_parts")),
    ("compute_node_fa", ("fa_bucket_define", "fa_submit", "fa_finalize")),  # section 5
])
def test_integration_binding_compiles(tmp_path, name, syms):
    import torch
    tdir = os.path.dirname(torch.__file__)
    src = tmp_path / (name + ".cpp")
    src.write_text(snippet(name))
    inc = ["-I" + os.path.join(REF, d) for d in ("pipeline_simulation", "pipeline_simulation/profiling", "models", "models/vgg", "models/resnet",
                                                 "models/lenet5", "datasets", "utils")]
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-w", "-D_GLIBCXX_USE_CXX11_ABI=1", "-I" + os.path.join(ROOT, "include")]
    cmd += inc + ["-isystem", os.path.join(tdir, "include"), "-isystem",
                  os.path.join(tdir, "include", "torch", "csrc", "api", "include"), str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    # the binding uses the ABI it documents
    for sym in syms:
        assert sym + "(" in snippet(name)
