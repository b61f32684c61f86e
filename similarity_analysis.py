"""Statistical similarity of the per-epoch synthetic tables (CLI of `Server/similarity_analysis.py:88-118`).

    python similarity_analysis.py -nepoch 500
writes ``{name}_statistical_similarity_analysis.csv`` with columns
``Epoch_No., Avg_JSD, Avg_WD, time_stamp`` (time_stamp = cumulative round time from
``timestamp_experiment.csv``).  Extra flags select another dataset / result directory.
"""
import argparse
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fed_tgan_amd.data.schema import get_spec  # noqa: E402
from fed_tgan_amd.eval.similarity import similarity_table, stat_sim_normalize  # noqa: E402,F401


if not sys.warnoptions:          # as the reference scripts do
    warnings.simplefilter("ignore")


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-nepoch", help="number of training epoch", required=True)
    p.add_argument("-config", default="intrusion")
    p.add_argument("-real_path", default=None)
    p.add_argument("-result_dir", default=None)
    p.add_argument("-timestamps", default="timestamp_experiment.csv")
    p.add_argument("-out", default=None)
    args = p.parse_args(argv)
    spec = get_spec(args.config)
    real = args.real_path or f"data/raw/{spec.name}_train.csv"
    rdir = args.result_dir or f"{spec.name}_result"
    fakes = [os.path.join(rdir, f"{spec.name}_synthesis_epoch_{i}.csv") for i in range(int(args.nepoch))]
    ts = args.timestamps if os.path.exists(args.timestamps) else None
    df = similarity_table(real, fakes, spec.categorical_list, ts)
    out = args.out or f"{spec.name}_statistical_similarity_analysis.csv"
    df.to_csv(out, index=False)
    print(df.tail().to_string(index=False))


if __name__ == "__main__":
    main()
