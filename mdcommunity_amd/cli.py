"""Command-line drop-in for the reference's test scripts (``run.sh`` dispatches here).

    python -m mdcommunity_amd.cli unit   testSynthetic --output DIR   # U/testSynthetic.py
    python -m mdcommunity_amd.cli unit   testReal      --output DIR   # U/testReal.py
    python -m mdcommunity_amd.cli degree testSynthetic --output DIR   # D/testSynthetic.py
    python -m mdcommunity_amd.cli degree testReal      --output DIR   # D/testReal.py

Same inputs and outputs as the reference scripts: testSynthetic reads
``<data-root>/synthetic/<type>/syn_<N>/adj{1,2}_<i>.npy`` and writes
``<output><type>/result_<N>_unit_cost.txt`` with ``'%.4f±%.2f,'``; testReal reads
``<data-root>/real/<name>.edges`` and writes the harness files of EvaluateRealData plus
``StepRatio_<r>/time&audc_<name>.csv``.  Defaults are the reference scripts' own lists
(U/testReal.py:24-66, D/testReal.py:24-60, U/testSynthetic.py:14-20); the rollouts run on the
GPU through libmdroll.so.  Training (``train``, ``drawLmcc``) is out of scope.
"""
import argparse
import os
import sys

import numpy as np

UNIT_SYN_MODEL = "./models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt"   # U/testSynthetic.py:19
UNIT_REAL_MODEL = "./models/g0-1_10w_TORCH-Model_GMM_30_50/nrange_30_50_iter_24000.ckpt"  # U/testReal.py:78-79
DEGREE_MODEL = "./models/nrange_30_50_iter_100000.ckpt"                                   # D/testReal.py:79
SYN_SIZES = ["32", "64", "128", "256", "512", "1024"]
SYN_TYPES = ["data_g", "data_gamma", "data_k"]
# (name, N, layers) as enabled in the reference scripts
UNIT_REAL = [("Padgett-Florentine-Families_multiplex", 16, (1, 2)),
             ("netsci_co-authorship_multiplex", 1400, (1, 2)),
             ("Lazega-Law-Firm_multiplex", 71, (1, 3))]
DEGREE_REAL = [("fao_trade_multiplex", 214, (3, 24))]


def _agent(variant):
    if variant == "degree":
        from .agent_degree import MultiDismantler
    else:
        from .agent import MultiDismantler
    return MultiDismantler()


def _dataset(spec):
    name, n, layers = spec.split(":")
    l0, l1 = layers.split(",")
    return name, int(n), (int(l0), int(l1))


def test_synthetic(variant, output, data_root, sizes, types, model=None):
    dqn = _agent(variant)
    model_file = model or (DEGREE_MODEL if variant == "degree" else UNIT_SYN_MODEL)
    lines = {}
    for data_type in types:
        file_path = output + data_type
        if not os.path.exists(file_path):
            os.makedirs(file_path)
        for n in sizes:
            with open("%s/result_%s_unit_cost.txt" % (file_path, n), "w") as fout:
                score_mean, score_std, _, _, _ = dqn.Evaluate(None, n, data_type, model_file, data_root=data_root)
                line = "%.4f±%.2f," % (score_mean, score_std)
                fout.write(line)
                lines[(data_type, n)] = line
                print("data_test_%s has been tested!" % n)
    return lines


def test_real(variant, output, data_root, datasets, step_ratio=0.0, model=None):
    import pandas as pd
    dqn = _agent(variant)
    model_file = model or (DEGREE_MODEL if variant == "degree" else UNIT_REAL_MODEL)
    save_dir = output
    if not os.path.exists(save_dir):
        os.makedirs(save_dir, exist_ok=True)
    print("The best model is :%s" % model_file)
    dqn.LoadModel(model_file)
    names = [d[0] for d in datasets]
    out = {}
    for j, (name, n, layers) in enumerate(datasets):
        df = pd.DataFrame(np.arange(2 * len(names)).reshape((2, len(names))), index=["time", "score"], columns=names)
        print("\nTesting dataset %s" % name)
        solution, t, score = dqn.EvaluateRealData(model_file, name + ".edges", save_dir, step_ratio, n, layers,
                                                  data_root=data_root)
        # the reference's int64 frame takes floats in column j (pandas upcasts it to float64)
        df[df.columns[j]] = df[df.columns[j]].astype(np.float64)
        df.iloc[0, j] = t
        df.iloc[1, j] = score
        print("Data:%s, time:%.2f, audc:%.6f" % (name, t, score))
        save_dir_local = save_dir + "/StepRatio_%.4f" % step_ratio
        if not os.path.exists(save_dir_local):
            os.mkdir(save_dir_local)
        df.to_csv(save_dir_local + "/time&audc_%s.csv" % name, encoding="utf-8", index=False)
        out[name] = (solution, t, score)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mdcommunity_amd.cli", description=__doc__.split("\n\n")[0])
    ap.add_argument("variant", choices=["unit", "degree"])
    ap.add_argument("command", choices=["testSynthetic", "testReal", "train", "drawLmcc"])
    ap.add_argument("-o", "--output", required=True, help="path to output file")
    ap.add_argument("--data-root", default="../../data", help="directory holding synthetic/ and real/")
    ap.add_argument("--model", default=None, help="checkpoint (reference path or .npz)")
    ap.add_argument("--sizes", default=",".join(SYN_SIZES))
    ap.add_argument("--types", default=",".join(SYN_TYPES))
    ap.add_argument("--dataset", action="append", default=None, help="name:N:l1,l2 (repeatable)")
    ap.add_argument("--step-ratio", type=float, default=0.0)
    a = ap.parse_args(argv)
    if a.command in ("train", "drawLmcc"):
        print("%s is not part of the MI355X inference engine (training and plotting are out of scope)" % a.command)
        return 2
    if a.command == "testSynthetic":
        test_synthetic(a.variant, a.output, a.data_root, a.sizes.split(","), a.types.split(","), a.model)
    else:
        ds = [_dataset(s) for s in a.dataset] if a.dataset else (DEGREE_REAL if a.variant == "degree" else UNIT_REAL)
        test_real(a.variant, a.output, a.data_root, ds, a.step_ratio, a.model)
    return 0


if __name__ == "__main__":
    sys.exit(main())
