"""CPU restatement vs the reference itself, timed on the same cores: the oracle
(oracle/torch_ref.py, the GPU box's CPU baseline) and the reference SeparationModel imported through the
offline stand-ins of tests/golden/make_golden.py, same weights, same B=64 x N=32000 inputs.
Runs in the build container only (the reference does not exist on the GPU box).

    python tools/cpu_ratio.py [threads]
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def timeit(fn, x, reps=3):
    fn(x[:2])
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn(x)
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    from make_golden import build, import_reference
    from oracle.torch_ref import OracleModel
    import sep_tfanet_vad_amd as pkg
    from sep_tfanet_vad_amd import synth
    ref_model, _, _ = import_reference()
    cfg = pkg.CONFIG_WITH_VAD
    net, sd = build(ref_model, cfg)
    om = OracleModel(cfg, {k: torch.from_numpy(v) for k, v in sd.items()}, torch.float32)
    x = torch.from_numpy(synth.make_batch(64, 32000, 7000)[0])
    with torch.no_grad():
        t_ref = timeit(lambda v: net(v), x)
        t_or = timeit(lambda v: om(v), x)
        d = (net(x[:4])[0] - om(x[:4])[0]).abs().max().item()
    print(f"threads={threads} B=64 N=32000: reference {64 / t_ref:.1f} utt/s ({t_ref:.3f} s), "
          f"oracle restatement {64 / t_or:.1f} utt/s ({t_or:.3f} s), ratio oracle/reference "
          f"{t_ref / t_or:.3f} (throughput); sep max-abs oracle vs reference {d:.2e}")


if __name__ == "__main__":
    main()
