"""Centralised (single-site) CTGAN synthesizer API.

Parity with ``CTGANSynthesizer`` / ``BaseSynthesizer`` (`Server/dtds/synthesizers/ctgan.py:309-488`,
`Server/dtds/synthesizers/base.py:6-30`): same hyper-parameters (embedding 128, G/D (256, 256),
l2scale 1e-6, batch 500, epochs), ``fit(train_data, categorical_columns, ordinal_columns)``
and ``sample(n)`` returning decoded rows, printing ``EPOCH i: loss_d loss_g time`` per epoch.
Training runs on :class:`~fed_tgan_amd.models.engine.CTGANEngine` (HIP kernels + hipGraph on a
GPU, eager torch ops on the CPU) instead of the reference's autograd loop.
"""
from __future__ import annotations

import time
from typing import Optional, Sequence

import numpy as np
import torch

from ..features.transformer import VGMTransformer
from .engine import CTGANEngine, EngineConfig
from .samplers import CondTables


class BaseSynthesizer:
    """SDGym-style base class: ``fit`` + ``sample`` (+ ``fit_sample``)."""

    def fit(self, data, categorical_columns=tuple(), ordinal_columns=tuple()):
        raise NotImplementedError

    def sample(self, samples: int):
        raise NotImplementedError

    def fit_sample(self, data, categorical_columns=tuple(), ordinal_columns=tuple()):
        self.fit(data, categorical_columns, ordinal_columns)
        return self.sample(data.shape[0])


class CTGANSynthesizer(BaseSynthesizer):
    def __init__(self, embedding_dim: int = 128, gen_dim: Sequence[int] = (256, 256), dis_dim: Sequence[int] = (256, 256),
                 l2scale: float = 1e-6, batch_size: int = 500, epochs: int = 3, device: Optional[str] = None,
                 backend: str = "auto", precision: str = "bf16", gmm_backend: str = "sklearn", seed: Optional[int] = None,
                 verbose: bool = True):
        self.embedding_dim = embedding_dim
        self.gen_dim = tuple(gen_dim)
        self.dis_dim = tuple(dis_dim)
        self.l2scale = l2scale
        self.batch_size = batch_size
        self.epochs = epochs
        self.device = torch.device(device or ("cuda:0" if torch.cuda.is_available() else "cpu"))
        self.backend = backend
        self.precision = precision
        self.gmm_backend = gmm_backend
        self.seed = seed
        self.verbose = verbose
        self.transformer: Optional[VGMTransformer] = None
        self.engine: Optional[CTGANEngine] = None
        self.history = []

    def fit(self, train_data, categorical_columns=tuple(), ordinal_columns=tuple()):
        rng = np.random.default_rng(self.seed)
        self.transformer = VGMTransformer().fit(np.asarray(train_data), categorical_columns, ordinal_columns,
                                                backend=self.gmm_backend, seed=self.seed, device=self.device)
        enc = self.transformer.transform(np.asarray(train_data), rng)
        cfg = EngineConfig(embedding_dim=self.embedding_dim, gen_dims=self.gen_dim, dis_dims=self.dis_dim,
                           batch_size=self.batch_size, l2scale=self.l2scale, precision=self.precision)
        self.engine = CTGANEngine(self.transformer.layout, cfg, self.device, backend=self.backend, seed=self.seed)
        self.engine.set_training_data(enc)
        self._cond_counts = CondTables.span_counts(enc, self.transformer.layout)
        self.engine.set_generation_tables(CondTables(self.transformer.layout, self._cond_counts), self.transformer)
        for i in range(self.epochs):
            t = time.time()
            self.engine.train_epoch()
            ld, lg = self.engine.losses()
            self.history.append((ld, lg))
            if self.verbose:
                print(f"EPOCH {i}:   loss_d:{ld:>6.2f}   loss_g:{lg:>6.2f}   time taken: {time.time() - t:.2f} sec")
        return self

    def sample(self, n: int) -> np.ndarray:
        """Decoded rows (continuous values and categorical labels as in ``transformer.inverse_transform``)."""
        return self.engine.generate_decoded(n).cpu().numpy()

    def sample_encoded(self, n: int) -> np.ndarray:
        return self.engine.generate_encoded(n).cpu().numpy()

    def save(self, path: str):
        """Model bundle (the reference's unused ``save_model``, `Server/dtds/distributed.py:560-563`,
        pickles ``[G, cond, transformer, batch_size, embedding_dim]``).  Here: plain tensors and
        Python containers only, so :meth:`load` reads it with ``weights_only=True``."""
        eng = self.engine
        torch.save({"G": eng.g_state_dict(), "D": eng.d_state_dict(), "transformer": self.transformer.to_dict(),
                    "cond_counts": torch.as_tensor(self._cond_counts),
                    "config": {"embedding_dim": self.embedding_dim, "gen_dim": list(self.gen_dim),
                               "dis_dim": list(self.dis_dim), "batch_size": self.batch_size, "l2scale": self.l2scale,
                               "epochs": self.epochs}}, path)

    @classmethod
    def load(cls, path: str, device: Optional[str] = None, backend: str = "auto") -> "CTGANSynthesizer":
        blob = torch.load(path, map_location="cpu", weights_only=True)
        c = blob["config"]
        syn = cls(embedding_dim=c["embedding_dim"], gen_dim=c["gen_dim"], dis_dim=c["dis_dim"], l2scale=c["l2scale"],
                  batch_size=c["batch_size"], epochs=c["epochs"], device=device, backend=backend, verbose=False)
        syn.transformer = VGMTransformer.from_dict(blob["transformer"])
        cfg = EngineConfig(embedding_dim=syn.embedding_dim, gen_dims=syn.gen_dim, dis_dims=syn.dis_dim,
                           batch_size=syn.batch_size, l2scale=syn.l2scale, precision=syn.precision)
        syn.engine = CTGANEngine(syn.transformer.layout, cfg, syn.device, backend=backend)
        syn.engine.load_g_state_dict(blob["G"])
        syn.engine.load_d_state_dict(blob["D"])
        syn._cond_counts = blob["cond_counts"].numpy()
        syn.engine.set_generation_tables(CondTables(syn.transformer.layout, syn._cond_counts), syn.transformer)
        return syn
