"""Host-side profile of the design-matrix step on the GPU box (development tool): cProfile of
bench.py's designmat step, to separate the host's launch / plan time from the kernels."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import torch
    import bench
    from sglm_hip import designmat, synth
    states = ["Select", "Consumption", "ENLP"]
    ts, tr = synth.designmat_session(bench.DM_TRIALS, 300)
    n = len(ts)
    tri = tr.set_index("nTrial").convert_dtypes()
    cols, dts = designmat.upload(ts, states)

    def step():
        return designmat.design_matrix_device(cols, dts, n, tri, states, [1],
                                              bench.DM_INTERACTIONS, verbose=False)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        step()
    host = (time.perf_counter() - t) / 10
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / 10
    print(f"host enqueue {host * 1e3:.3f} ms/step, wall {wall * 1e3:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
