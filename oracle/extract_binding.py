#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: writes the reference-side binding block `// <name>.cpp ...` of INTEGRATION.md,
verbatim, to the given path (oracle/Makefile.ref compiles it into oracle/_ref/ref_aggregator).

  python3 oracle/extract_binding.py aggregator_fa oracle/_ref/aggregator_fa.cpp
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def block(name):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```cpp\n(// %s\.cpp.*?)```" % re.escape(name), text, re.S)
    if not m:
        sys.exit("INTEGRATION.md binding block %s not found" % name)
    return m.group(1)


if __name__ == "__main__":
    name, out = sys.argv[1], sys.argv[2]
    src = block(name)
    if not os.path.exists(out) or open(out).read() != src:  # keep make's timestamps when unchanged
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as f:
            f.write(src)
