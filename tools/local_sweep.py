"""The local mode's kernel at one shape under several launch settings, in ONE process (the C5
shape's 1.5e8 positives are generated and uploaded once): per variant, a warm-up and a timed
region of whole 128-step periods, step time by the library's live HIP events, algorithmic TB/s
and the fraction of the 8 TB/s roofline.  Variants are environment settings
the library reads at every launch (hogwild.hip: BPRMF_HOGWILD_WINDOW; the other round-4 launch
knobs were removed in round 6 with their measured settings fixed).

  python tools/local_sweep.py [--shape c5|ml20m] [--steps 1024] "NAME:ENV=v,ENV=v" ...
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"c5": (10_000_000, 100_000_000, 150_000_000, 256),
          "ml20m": (138493, 26744, 10_000_000, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="c5", choices=sorted(SHAPES))
    ap.add_argument("--steps", type=int, default=1024)
    ap.add_argument("--warmup", type=int, default=256)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch
    rl = importlib.import_module("recommend-lib_amd")
    syn = importlib.import_module("recommend-lib_amd.synthetic")
    U, I, npos, d = SHAPES[a.shape]
    B = 4096
    t0 = time.time()
    pos = syn.make_positives(U, I, npos, 20261015)
    print(f"# {a.shape}: {len(pos)} positives in {time.time() - t0:.0f} s", flush=True)
    m = rl.BPRMF(U, I, d, lr=0.01, wd=0.001, batch_size=B, num_ng=4, seed=20261015, device=0,
                 semantics="local", local_steps=128)
    m.set_train(pos)
    del pos
    n_steps = m.epoch_size()[1]
    at = [0]

    def run(k):
        done = 0
        while done < k:
            e, s = divmod(at[0], n_steps)
            c = min(k - done, n_steps - s)
            m.train_steps(e, s, c)
            done += c
            at[0] += c

    base = dict(os.environ)
    bpt = 24 * d + 12
    for rep in range(a.reps):
        for spec in a.variants:
            name, _, envs = spec.partition(":")
            os.environ.clear()
            os.environ.update(base)
            for kv in filter(None, envs.split(",")):
                k, v = kv.split("=", 1)
                os.environ[k] = v
            run(a.warmup)
            torch.cuda.synchronize()
            m.profile(True)
            w0 = time.perf_counter()
            run(a.steps)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - w0) / a.steps * 1e6
            kp = m.profile_read()
            m.profile(False)
            us = kp["step_graph"]["ms"] / kp["step_graph"]["count"] * 1e3
            tbs = B * bpt / (us * 1e-6) / 1e12
            print(json.dumps(dict(shape=a.shape, variant=name, rep=rep, env=envs, us_per_step=round(us, 3),
                                  wall_us_per_step=round(wall, 3), tb_s=round(tbs, 3),
                                  frac=round(tbs / 8.0, 4))), flush=True)
    os.environ.clear()
    os.environ.update(base)


if __name__ == "__main__":
    main()
