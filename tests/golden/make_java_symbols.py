#!/usr/bin/env python3
"""The reference's declarations (every class of minijava/src: fields,
methods with arity / static-ness / return type / visibility, constructors,
extends / implements) into tests/golden/java_symbols.json, the table
tests/test_java_refs.py resolves the Java drop-ins' member uses against.

Run here, where /root/reference exists (the GPU box has no reference):
    python3 tests/golden/make_java_symbols.py [/root/reference/minijava/src]
The JSON is data extracted by tests/javarefs.symbols (no source text)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import javarefs  # noqa: E402


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/minijava/src"
    table = javarefs.tree_symbols(src)
    for rec in table.values():
        rec["source"] = "R/" + rec["source"]
    path = os.path.join(HERE, "java_symbols.json")
    with open(path, "w") as f:
        json.dump(table, f, sort_keys=True, separators=(",", ":"))
        f.write("\n")
    print(path, len(table), "classes")


if __name__ == "__main__":
    main()
