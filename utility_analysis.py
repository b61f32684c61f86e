"""ML utility of a synthetic table (CLI of `Server/utility_analysis.py:94-119`).

    python utility_analysis.py -train_path data/raw/Intrusion_train.csv \
        -test_path data/raw/Intrusion_test.csv -synthetic_path Intrusion_result/Intrusion_synthesis_epoch_0.csv
prints the real-minus-synthetic [accuracy, weighted F1] matrix of LR / DT / RF / MLP and the
mean F1 difference.
"""
import argparse
import os
import sys
import warnings

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fed_tgan_amd.data.schema import get_spec  # noqa: E402
from fed_tgan_amd.eval.utility import real_res  # noqa: E402


if not sys.warnoptions:          # as the reference scripts do
    warnings.simplefilter("ignore")


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-train_path", default="data/raw/Intrusion_train.csv", help="path to train dataset")
    p.add_argument("-test_path", default="data/raw/Intrusion_test.csv", help="path to test dataset")
    p.add_argument("-synthetic_path", default="Intrusion_result/Intrusion_synthesis_epoch_0.csv",
                   help="path to synthetic dataset")
    p.add_argument("-config", default="intrusion")
    args = p.parse_args(argv)
    spec = get_spec(args.config)
    real = pd.read_csv(args.train_path)
    test = pd.read_csv(args.test_path)
    fake = pd.read_csv(args.synthetic_path)
    original_real = pd.concat([real, test])
    print("=========== evaluation for real data===============")
    real_utility = real_res(original_real, real, test, spec.target_column, spec.categorical_list)
    print("=========== evaluation for synthetic data===============")
    fake_utility = real_res(original_real, fake, test, spec.target_column, spec.categorical_list)
    diff = np.array(real_utility) - np.array(fake_utility)
    f1 = float(diff.mean(axis=0)[1])
    print("difference in accuracy and f1-score for all AL algorithms: ", diff)
    print("difference in f1-score: ", f1)
    return diff, f1


if __name__ == "__main__":
    main()
