"""Centralised CTGANSynthesizer API (fit / sample) and reference-layout state dicts."""
import numpy as np
import torch

from fed_tgan_amd.models.ctgan import Discriminator, Generator
from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
from fed_tgan_amd.models.synthesizer import CTGANSynthesizer

from helpers import small_table


def test_fit_and_sample_cpu(tmp_path):
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    syn = CTGANSynthesizer(epochs=2, batch_size=100, device="cpu", verbose=False, seed=0)
    syn.fit(enc[:800], tp.categorical_indices())
    out = syn.sample(300)
    assert out.shape == (300, enc.shape[1]) and np.isfinite(out).all()
    cat = tp.categorical_indices()
    for j in cat:   # sampled categories are valid label codes of the column
        assert set(np.unique(out[:, j])) <= set(np.unique(enc[:800, j]))
    assert len(syn.history) == 2
    syn.save(str(tmp_path / "m.pt"))


def test_state_dict_roundtrip_with_reference_modules():
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    eng = CTGANEngine(tr.layout, EngineConfig(batch_size=100), "cpu", backend="torch")
    G, D = eng.to_modules()
    assert isinstance(G, Generator) and isinstance(D, Discriminator)
    sd = G.state_dict()
    assert "seq.0.fc.weight" in sd and "seq.1.bn.running_var" in sd and "seq.2.weight" in sd
    assert set(D.state_dict()) == {"seq.0.weight", "seq.0.bias", "seq.3.weight", "seq.3.bias", "seq.6.weight",
                                   "seq.6.bias"}
    eng2 = CTGANEngine(tr.layout, EngineConfig(batch_size=100), "cpu", backend="torch")
    eng2.load_modules(G, D)
    assert torch.equal(eng.flat, eng2.flat)
    # the engine's generator forward (eval) equals the reference module's forward
    G.eval()
    x = torch.randn(64, eng.E + eng.C)
    H = torch.zeros(64, eng.Hw)
    H[:, eng.off[0]:] = x
    logits = torch.zeros(64, eng.Dd)
    eng._g_forward(H, logits, training=False, nhat=False)
    assert torch.allclose(logits, G(x), atol=1e-5)


def test_save_load_roundtrip(tmp_path):
    """save() writes plain tensors/containers; load() reads them back with weights_only=True."""
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    syn = CTGANSynthesizer(epochs=1, batch_size=100, device="cpu", verbose=False, seed=0)
    syn.fit(enc[:800], tp.categorical_indices())
    p = str(tmp_path / "m.pt")
    syn.save(p)
    again = CTGANSynthesizer.load(p, device="cpu")
    for k, v in syn.engine.g_state_dict().items():
        assert torch.equal(v, again.engine.g_state_dict()[k]), k
    assert again.transformer.output_info == syn.transformer.output_info
    out = again.sample(200)
    assert out.shape == (200, enc.shape[1]) and np.isfinite(out).all()


def test_grad_flow_report(tmp_path):
    from fed_tgan_amd.utils.gradflow import GradFlow
    spec, df, tp, meta, vocabs, enc, tr, X = small_table()
    eng = CTGANEngine(tr.layout, EngineConfig(batch_size=100), "cpu", backend="torch")
    eng.set_training_data(X)
    gf = GradFlow()
    for _ in range(2):
        eng.train_steps(2, use_graph=False)
        gf.update(eng)
    assert gf.layers["D"][0] == "seq.0.weight" and len(gf.ave["G"]) == 2
    # every weight gets gradient (the D output bias's WGAN gradient is exactly 0: seeds sum to 0)
    assert all(v > 0 for n, v in zip(gf.layers["D"], gf.ave["D"][-1]) if n.endswith("weight"))
    gf.save_csv(str(tmp_path / "gf.csv"))
    assert (tmp_path / "gf.csv").stat().st_size > 0
    gf.plot(str(tmp_path))


def test_dtds_local_cli(tmp_path):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = [sys.executable, "-m", "dtds.local", "-rows", "2000", "-epochs", "1", "-batch_size", "100", "-n_sample",
            "300", "-report", "-gmm", "torch", "-backend", "torch", "-out_dir", str(tmp_path)]
    r = subprocess.run(args, cwd=root, env=dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="2"),
                       capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    rep = tmp_path / "reports" / "Intrusion_epoch1"
    assert (rep / "column_similarity.csv").exists() and (rep / "Intrusion_synthetic.csv").exists()
