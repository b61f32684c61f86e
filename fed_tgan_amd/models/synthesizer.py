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
        self.engine.set_generation_tables(CondTables.from_encoded(enc, self.transformer.layout), self.transformer)
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
        """Model bundle (the reference's unused ``save_model``, `Server/dtds/distributed.py:560-563`)."""
        torch.save({"G": self.engine.g_state_dict(), "D": self.engine.d_state_dict(),
                    "layout": self.transformer.output_info, "bank": self.transformer.bank.to_dict(),
                    "components": self.transformer.components.tolist(), "meta": self.transformer.meta,
                    "config": {"embedding_dim": self.embedding_dim, "gen_dim": self.gen_dim, "dis_dim": self.dis_dim,
                               "batch_size": self.batch_size}}, path)
