#!/usr/bin/env python3
"""Extract the public API (constructors, methods, fields) of the reference
classes the Java drop-ins mirror into tests/golden/java_api.json.

Run here, where /root/reference exists (the GPU box has no reference):
    python3 tests/golden/make_java_api.py [/root/reference/minijava/src]

The committed JSON is data (class -> signatures: parameter types with array
brackets normalised, `final` dropped); tests/test_java_api.py parses the
drop-ins under java/ with the same parser (javaapi.py) and asserts that each
declares every signature of its reference class.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import javaapi  # noqa: E402

# reference class (package/File.java) -> drop-in (java/package/File.java)
MIRRORED = {
    "iterator/ColumnarFileScan.java": "iterator/GpuColumnarFileScan.java",
    "iterator/ColumnarColumnScan.java": "iterator/GpuColumnarColumnScan.java",
    "iterator/ColumnarColumnsScan.java": "iterator/GpuColumnarColumnsScan.java",
    "iterator/ColumnarNestedLoopJoins.java": "iterator/GpuColumnarNestedLoopJoins.java",
    "index/ColumnIndexScan.java": "index/GpuColumnIndexScan.java",
    "index/ColumnarIndexScan.java": "index/GpuColumnarIndexScan.java",
}


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/minijava/src"
    out = {}
    for ref, dropin in sorted(MIRRORED.items()):
        with open(os.path.join(src, ref)) as f:
            api = javaapi.public_api(f.read())
        api["source"] = "R/" + ref
        api["dropin"] = "java/" + dropin
        out[api.pop("class")] = api
    path = os.path.join(HERE, "java_api.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(path)


if __name__ == "__main__":
    main()
