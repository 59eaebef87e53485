"""Per-phase cycle breakdown of the replay kernel (profiling build, -DMT_PROF).

Builds fluidframework_amd/build/libmtreplay_prof.so, replays a config-3 batch on cuda:0 and prints
where each document's shader-clock cycles went (phases nest: HEAP inside ZAMBONI/MAP, SPLIT inside
FIND callers, etc.). Usage: python tools/phase_profile.py [--build-only] [--docs N]
"""
import argparse, ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fluidframework_amd import native

PHASES = ["APPLY", "ZAMBONI", "FIND", "MAP", "SPLIT", "ACK", "TEXT", "HEAP", "SCOUR", "PACK", "APPEND", "CAND", "S1load", "S2walk", "S3compact", "P1leaf", "P2interior", "INSROW", "LEAFINS",
          "WIN", "TFIND", "LFIND", "ROPE", "RESTAT", "VISIT", "PLACE",
          "#ins", "#range", "#winrows", "#winmiss", "#scour", "#pack",
          "#heapsize", "#pop", "#push"]
LIB = os.environ.get("MT_PROF_LIB") or native.lib_path("libmtreplay_prof.so")  # MT_PROF_LIB: a prebuilt copy


def build():
    native.build_replay(defines=("MT_PROF",), name="libmtreplay_prof.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--docs", type=int, default=2048)
    ap.add_argument("--ops", type=int, default=4096)
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    if a.build_only:
        build()
        return
    import numpy as np
    if not os.path.exists(LIB):  # kept out of the default push (.gpurunignore): built where it runs
        build()
    os.environ["MT_REPLAY_LIB"] = LIB
    from fluidframework_amd import gen
    from fluidframework_amd.engine import Engine, default_caps, lib
    w = {3: gen.config3, 4: gen.config4, 5: gen.config5, 2: gen.config2}[a.config](a.ops)
    b = gen.generate(w, a.docs)
    eng = Engine(b.ndocs, **default_caps(a.ops, config=a.config))
    eng.start_collab(b.local_long_id)
    eng.replay(b)
    L = lib()
    L.mt_engine_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    out = np.zeros((b.ndocs, len(PHASES)), np.uint64)
    assert L.mt_engine_profile(eng.h, out.ctypes.data) == 0
    tot = out.sum(0).astype(np.float64)
    ev = b.nops
    print(f"config {a.config} docs {b.ndocs} events {ev} kernel {eng.last_run_ms:.1f} ms")
    for i, n in enumerate(PHASES):
        if n.startswith("#"):  # event counts
            print(f"{n:8s} {tot[i] / ev:10.3f} per event")
        else:
            print(f"{n:8s} {tot[i] / ev:10.0f} cycles/event  {100 * tot[i] / tot[0]:5.1f}% of APPLY")
    ci, cr = tot[PHASES.index("#ins")], tot[PHASES.index("#range")]
    if ci and cr:
        print(f"per insert: INSROW {tot[PHASES.index('INSROW')] / ci:.0f} PLACE {tot[PHASES.index('PLACE')] / ci:.0f}; "
              f"per range op: MAP {tot[PHASES.index('MAP')] / cr:.0f} VISIT {tot[PHASES.index('VISIT')] / cr:.0f}")


if __name__ == "__main__":
    main()
