"""Motion ingestion throughput: he_ingest_clips on the GPU vs the host restatement
(numpy/scipy build_tables) on the same synthetic clips (§8d recipe), 4096 clips x 150 frames by
default (the reference took 188 s for this on its CPU path).

Usage: python tools/ingest_bench.py [--clips 4096] [--frames 150] [--host-sample 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=4096)
    ap.add_argument("--frames", type=int, default=150)
    ap.add_argument("--host-sample", type=int, default=256)
    a = ap.parse_args()
    import torch
    from humanoid_amd import synthetic
    from humanoid_amd.engine import Engine
    from humanoid_amd.model import load_default_model
    from humanoid_amd.motion_lib import build_tables
    model = load_default_model()
    rng = np.random.default_rng(0)
    base = [synthetic.make_clip(model, rng, num_frames=a.frames) for _ in range(16)]
    clips = [base[i % 16] for i in range(a.clips)]  # distinct clip objects are not needed for timing
    eng = Engine(model, 16, device=0)
    eng.ingest_clips(clips[:64])  # warm-up (allocation, code objects)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.ingest_clips(clips)
    torch.cuda.synchronize()
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    build_tables(model, clips[:a.host_sample])
    t_host = (time.perf_counter() - t0) * a.clips / a.host_sample
    frames = a.clips * a.frames
    print(json.dumps({"clips": a.clips, "frames": frames, "device_s": round(t_dev, 4),
                      "device_frames_per_s": round(frames / t_dev), "host_s_extrapolated": round(t_host, 2),
                      "host_sample_clips": a.host_sample, "speedup": round(t_host / t_dev, 1),
                      "note": "device time includes the H2D copy of the clip arrays and table allocation"}))


if __name__ == "__main__":
    main()
