"""Element stiffness / mass kernel timing on the BASELINE configs[4] families (c3d8 88^3, c3d6 2*70^3, c3d10 6*48^3,
jittered): best of 5 event-timed calls of compute_K_matrix / compute_M_matrix after a warm-up, output write GB/s,
and a checksum of the element matrices (build variants must agree bit for bit). Select a library build with
FEM355_LIB=... (tools/build_variants.sh).

    python tools/iso_ke_probe.py
"""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fem355 import _capi as C, element, mesh  # noqa: E402

E, NU, RHO = 113.8e9, 0.342, 4.47e-3
FAMILIES = (("c3d8", mesh.hex_box, 88), ("c3d6", mesh.wedge_box, 70), ("c3d10", mesh.tet10_cube, 48))


def best_ms(fn, reps=5):
    best, out = None, None
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e)
        best = t if best is None else min(best, t)
    return best, out


def main():
    C.lib()
    dev = torch.device("cuda", 0)
    res = {"lib": os.environ.get("FEM355_LIB", "default")}
    for et, gen, n in FAMILIES:
        c, el = gen(n, jitter=0.1, device=dev)
        r = {}
        for name, fn in (("K", lambda: element.compute_K_matrix(c, el, et, E, NU, device=dev, dtype=torch.float64)),
                         ("M", lambda: element.compute_M_matrix(c, el, et, RHO, device=dev, dtype=torch.float64))):
            fn()
            ms, out = best_ms(fn)
            h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
            r[name] = {"ms": round(ms, 3), "write_GBps": round(out.numel() * 8 / ms / 1e6, 1), "sha1": h}
            del out
        res[et] = r
        print(et, json.dumps(r), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
