"""``python -m dtds.local`` -- standalone (centralised, single-site) CTGAN training + report.

The reference's `Server/dtds/local.py:1-48` is broken: it imports the nonexistent
`dtds.data.load.load_dataset` and `dtds.eval.distribution_analysis`. This is the working
equivalent on this framework's engine.

1. Load the table: `-datapath` CSV, or the named schema's synthetic generator.
2. Encode it with the reference's meta / label-encoder rules.
3. Train `CTGANSynthesizer` for `-epochs`.
4. Save `models/synthesizer_{name}_epoch{E}.pt`. Without `-report` it always trains; with
   `-report` it reuses that file when it already exists.
5. With `-report`, sample `-n_sample` rows, decode them to the original labels, and write
   `reports/{name}_epoch{E}/` with the synthetic CSV and the per-column JSD/WD table (the
   `similarity_analysis.py` metrics).

    python -m dtds.local -dataset intrusion -epochs 3 -report
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-dataset", default="intrusion", help="schema name (intrusion, adult, covertype, wide) or spec JSON")
    ap.add_argument("-datapath", default=None, help="training CSV (default: the schema's synthetic generator)")
    ap.add_argument("-rows", type=int, default=40000, help="synthetic rows when no -datapath")
    ap.add_argument("-epochs", default=3, type=int)
    ap.add_argument("-batch_size", default=500, type=int)
    ap.add_argument("-n_sample", default=1000, type=int)
    ap.add_argument("-report", action="store_true")
    ap.add_argument("-out_dir", default=".")
    ap.add_argument("-backend", default="auto")
    ap.add_argument("-gmm", default="sklearn")
    ap.add_argument("-seed", type=int, default=0)
    args = ap.parse_args(argv)

    import pandas as pd

    from fed_tgan_amd.data.decode import decode_frame
    from fed_tgan_amd.data.schema import get_spec
    from fed_tgan_amd.data.synthetic import generate
    from fed_tgan_amd.data.table import TablePreprocessor
    from fed_tgan_amd.eval.similarity import column_similarity
    from fed_tgan_amd.fed.stats import merge_categorical_metas
    from fed_tgan_amd.models.synthesizer import CTGANSynthesizer

    spec = get_spec(args.dataset)
    df = pd.read_csv(args.datapath) if args.datapath else generate(spec, args.rows, seed=args.seed)
    df = df[spec.selected_variables]
    tp = TablePreprocessor(df, f"{spec.name}_train", spec.problem_type,
                           "" if spec.target_column == "none" else spec.target_column, spec.categorical_list,
                           spec.nonnegative_list, spec.date_dic)
    meta, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    train = tp.encode(vocabs)
    cat_idx = tp.categorical_indices()

    name = f"{spec.name}_epoch{args.epochs}"
    mdir = os.path.join(args.out_dir, "models")
    os.makedirs(mdir, exist_ok=True)
    model_path = os.path.join(mdir, f"synthesizer_{name}.pt")
    if os.path.exists(model_path) and args.report:
        syn = CTGANSynthesizer.load(model_path, backend=args.backend)
    else:
        syn = CTGANSynthesizer(epochs=args.epochs, batch_size=args.batch_size, backend=args.backend,
                               gmm_backend=args.gmm, seed=args.seed)
        syn.fit(train, cat_idx)
        syn.save(model_path)
        print(f"saved {model_path}")

    if args.report:
        fake = decode_frame(syn.sample(args.n_sample), meta, vocabs)
        real = decode_frame(train, meta, vocabs)
        rdir = os.path.join(args.out_dir, "reports", name)
        os.makedirs(rdir, exist_ok=True)
        fake.to_csv(os.path.join(rdir, f"{spec.name}_synthetic.csv"), index=False)
        table = column_similarity(real, fake, spec.categorical_list)
        table.to_csv(os.path.join(rdir, "column_similarity.csv"), index=False)
        print(fake.head())
        print(table.to_string(index=False))
        print(f"report written to {rdir}")


if __name__ == "__main__":
    main()
