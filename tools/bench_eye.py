#!/usr/bin/env python3
"""Eye-tracking front end timing on 1 x MI355X: one
640x400 eye frame through RITnet (random weights of the reference's shapes;
the checkpoint is not in this repository), the pupil centroid and the fovea
mapping, next to the CPU oracle (torch float32 on the host cores) of the
same network.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import ritnet_oracle as R
    from gaussian_splatting_with_eye_tracking_amd import eye_tracking as E
    g = np.load(os.path.join(ROOT, "tests", "golden", "eye_pins.npz"))
    sd = R.random_state_dict(0)
    net = E.RITnet(sd)
    x = torch.from_numpy(E.preprocess(g["eye"])).cuda()
    for _ in range(3):
        net(x)
    torch.cuda.synchronize()
    reps = 50
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        _, labels = net(x)
    b.record()
    torch.cuda.synchronize()
    net_ms = a.elapsed_time(b) / reps
    E.track(net, g["eye"], (1920, 1080))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):  # host image in, fovea on the host out (upload, preprocess, network, centroid)
        labels, pxy, fovea = E.track(net, g["eye"], (1920, 1080))
    torch.cuda.synchronize()
    track_ms = (time.perf_counter() - t0) * 1e3 / reps
    E.preprocess(g["eye"])
    t0 = time.perf_counter()
    for _ in range(5):
        E.preprocess(g["eye"])
    pre_ms = (time.perf_counter() - t0) * 1e3 / 5
    gray = torch.from_numpy(g["eye"]).cuda()
    for _ in range(3):
        E.preprocess_device(gray)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        E.preprocess_device(gray)
    b.record()
    torch.cuda.synchronize()
    pre_dev_ms = a.elapsed_time(b) / reps
    t0 = time.perf_counter()
    R.forward(sd, E.preprocess(g["eye"]))
    cpu_ms = (time.perf_counter() - t0) * 1e3
    flops = 0
    for k, w in sd.items():
        if k.endswith(".weight") and w.dim() == 4:
            lvl = k.split(".")[0]
            n = int(lvl[-1]) if lvl.startswith("down_block") else (5 - int(lvl[-1])) if lvl.startswith("up_block") else 1
            px = (640 >> (n - 1)) * (400 >> (n - 1)) if lvl != "out_conv1" else 640 * 400
            flops += 2 * w.numel() * px
    from gaussian_splatting_with_eye_tracking_amd import _C

    _C.set_tuning("ritnet_mfma", 0)
    for _ in range(2):
        net(x)
    torch.cuda.synchronize()
    a.record()
    for _ in range(10):
        net(x)
    b.record()
    torch.cuda.synchronize()
    fma_ms = a.elapsed_time(b) / 10
    _C.set_tuning("ritnet_mfma", 1)
    print(json.dumps({"metric": "RITnet eye frames/s (640x400, fp32)", "ritnet_ms": round(net_ms, 4),
                      "ritnet_ms_vector_fma_kernel": round(fma_ms, 4),
                      "frames_per_s": round(1e3 / net_ms, 1), "gflop_per_frame": round(flops / 1e9, 2),
                      "achieved_tflops": round(flops / (net_ms * 1e-3) / 1e12, 2),
                      "track_ms": round(track_ms, 3), "device_preprocess_ms": round(pre_dev_ms, 4),
                      "host_preprocess_ms_numpy_restatement": round(pre_ms, 3),
                      "cpu_oracle_ms": round(cpu_ms, 1), "cpu_threads": torch.get_num_threads()}))


if __name__ == "__main__":
    main()
