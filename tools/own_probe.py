"""GPU probe: k_tbatch placements against the C restatement with KGPU_OPT_TBATCH_OWN 0 / 1, over the
persistent-topology test clusters at 2 workgroups (512 x 2) and the default geometry."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kubernetes-1_amd"))
if sys.argv[1:] == ["none"]:  # the committed build's package (_head/), placed first
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "_head", "kubernetes-1_amd"))
import numpy as np  # noqa: E402

import test_topo_persistent as T  # noqa: E402

OWNS = [None if v == "none" else int(v) for v in (sys.argv[1:] or ["0", "1", "0", "1"])]
for groups in (2, 0):
    for seed in range(8):
        line = []
        for own in OWNS:
            fw, w, got, rw, rg = T._run(T._big(seed), tfast=1, groups=groups, own=own)
            bad = np.nonzero(w["node"] != got["node"])[0]
            rows = sum(int(np.any(rw[k] != rg[k])) for k in rw)
            line.append("own%s:%d/%d%s" % (own, len(bad), rows, (" first %d" % bad[0]) if len(bad) else ""))
            fw.engine.close()
        print("groups %d seed %d  %s" % (groups, seed, "  ".join(line)), flush=True)
