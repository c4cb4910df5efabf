"""A/B of fit() at the reference's size (845 nodes, D = 64, R = 4, fold 0, HIP-graph replay) across variant
builds of libiddgcn_hip.so: ms per epoch of tools/train_folds.run, round-robin.
usage: python tools/ab_fit.py lib1.so lib2.so ... """
import sys

sys.path.insert(0, ".")
from iddgcn_amd import _lib as L  # noqa: E402
from tools.bench_mem import load_lenient  # noqa: E402
from tools.train_folds import run  # noqa: E402


def main(libs, epochs=1000, rounds=2):
    for _ in range(rounds):
        for lib in libs:
            L._lib = load_lenient(lib)
            r = run(0, 89, epochs)
            print(f"{lib:20s} {r['ms_per_epoch']:.3f} ms/epoch  auc {r['roc_auc']:.4f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
