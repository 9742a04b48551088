"""Minimal driver for rocprofv3 runs: renders the bench workloads through the
blocking C-ABI (smallpt 1920x1080 64 spp, Whitted 1920x1080) `reps` times."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "se-195-project-ray-tracer_amd"))
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--what", default="smallpt,whitted")
ap.add_argument("--spp", type=int, default=64)
a = ap.parse_args()
for _ in range(a.reps):
    if "smallpt" in a.what:
        rtamd.SmallptFrame(1920, 1080).render(a.spp)
    if "whitted" in a.what:
        rtamd.whitted_render(1920, 1080)
print("done")
