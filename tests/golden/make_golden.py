"""Regenerate tests/golden/*.json from the transcription modules (make_*.py).

Each make_*.py restates, as data, the table entries of one group of the reference's unit
tests; "src" is the reference file:line of the entry.  When /root/reference is readable the
line number is re-resolved from the case name (the file is only searched, never copied).
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
REF = "/root/reference"

GROUPS = ["noderesources", "tainttoleration", "nodeaffinity", "normalize", "generic", "node_tree",
          "podtopologyspread", "interpodaffinity", "defaultpodtopologyspread", "imagelocality",
          "nodepreferavoidpods", "nodeports", "nodename", "nodeunschedulable", "requestedtocapacityratio",
          "resourcelimits", "preemption", "framework", "misc"]


def resolve(cases):
    cache = {}
    for c in cases:
        f, _, line = c["src"].rpartition(":")
        path = os.path.join(REF, f)
        if not os.path.exists(path):
            continue
        if path not in cache:
            with open(path) as fh:
                cache[path] = fh.read().split("\n")
        lines = cache[path]
        pat = re.compile(r'name:\s*"%s"' % re.escape(c["name"]))
        hits = [i + 1 for i, ln in enumerate(lines) if pat.search(ln)]
        if hits:
            want = int(line) if line.isdigit() else 0
            c["src"] = "%s:%d" % (f, min(hits, key=lambda h: abs(h - want)))
    return cases


def main():
    for g in GROUPS:
        mod_path = os.path.join(HERE, "make_%s.py" % g)
        if not os.path.exists(mod_path):
            continue
        mod = __import__("make_%s" % g)
        cases = resolve(mod.all_cases())
        with open(os.path.join(HERE, "%s.json" % g), "w") as fh:
            json.dump(cases, fh, indent=1, sort_keys=True)
        print("%s: %d cases" % (g, len(cases)))


if __name__ == "__main__":
    main()
