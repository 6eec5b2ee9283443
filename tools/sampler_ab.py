#!/usr/bin/env python3
"""A/B of the host legacy-MT19937 sampler: libdopt.so's against an older build passed as
argv[1] (same C ABI), interleaved in one process, on the C3 and C2 shapes."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = {"new": ctypes.CDLL(os.path.join(ROOT, "distributed-optimization_amd", "libdopt.so")),
        "old": ctypes.CDLL(sys.argv[1])}


def run(lib, T, rows, b, adv=False):
    st = np.random.get_state()
    key = np.array(st[1], dtype=np.uint32)
    pos = ctypes.c_int32(st[2])
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    out = np.empty((T, len(rows), max(b, 1)), dtype=np.int32)
    vp = ctypes.c_void_p
    t = time.perf_counter()
    if adv:
        lib.dopt_mt_advance_rounds(vp(key.ctypes.data), ctypes.byref(pos), ctypes.c_int64(T), ctypes.c_int64(len(rows)),
                                   vp(rows.ctypes.data))
    else:
        lib.dopt_mt_choice_rounds(vp(key.ctypes.data), ctypes.byref(pos), ctypes.c_int64(T), ctypes.c_int64(len(rows)),
                                  vp(rows.ctypes.data), ctypes.c_int64(b), vp(out.ctypes.data))
    return time.perf_counter() - t


print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for name, T, rows, b in [("C3 b=m", 10, [512] * 4096, 1), ("C3 b=16", 10, [512] * 4096, 16), ("C2 b=16", 512, [500] * 25, 16)]:
    res = {"old": [], "new": [], "new-advance": []}
    for rep in range(5):
        np.random.seed(rep)
        res["old"].append(run(libs["old"], T, rows, b))
        res["new"].append(run(libs["new"], T, rows, b))
        if b == 1:
            res["new-advance"].append(run(libs["new"], T, rows, b, adv=True))
    draws = T * sum(r - 1 for r in rows)
    print(name, {k: f"{np.median(v) / draws * 1e9:.2f} ns/draw" for k, v in res.items() if v}, flush=True)
