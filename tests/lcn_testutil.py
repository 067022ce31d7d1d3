"""Shared helpers: build matching oracle / native configurations."""
import numpy as np

import lcn_oracle as O


def make_cfg(F=64, L=3, knn=3, mask="locally_connected", in_F=2, **kw):
    return O.Config(F=F, in_F=in_F, num_layers=L, mask_type=mask,
                    neighbour=O.neighbour_matrix(knn), **kw)


def mask_matrix(cfg):
    """What the C ABI takes: LC -> structure C (row = input joint), EXP -> 2^-d."""
    if cfg.learnable_mask:
        return O.structure(cfg)
    return O.exponential_matrix()


def make_network(cfg, max_batch, **kw):
    from lcn_amd.native import Network
    return Network(F=cfg.F, in_F=cfg.in_F, num_layers=cfg.num_layers, mask_type=cfg.mask_type,
                   mask_matrix=mask_matrix(cfg), residual=cfg.residual,
                   batch_norm=cfg.batch_norm, max_norm=cfg.max_norm,
                   regularization=cfg.regularization, learning_rate=cfg.learning_rate,
                   decay_steps=cfg.decay_steps, decay_rate=cfg.decay_rate, max_batch=max_batch,
                   **kw)


def perturbed_params(cfg, seed=1):
    """Kaiming init plus non-trivial BN affine and mask logits, so every
    gradient path is exercised (a fresh init has gamma=1, beta=0, V=N^T)."""
    p = O.init_params(cfg, seed)
    rng = np.random.default_rng(seed + 100)
    for k in p:
        if k.endswith("_gamma"):
            p[k] = (1.0 + 0.2 * rng.standard_normal(p[k].shape)).astype(np.float32)
        elif k.endswith("_beta"):
            p[k] = (0.1 * rng.standard_normal(p[k].shape)).astype(np.float32)
        elif k == "mask":
            p[k] = (p[k] + 0.3 * rng.standard_normal(p[k].shape)).astype(np.float32)
    return p


def synthetic_batch(B, in_F=2, seed=0):
    """x ~ U(-1,1) [B, 17*in_F]; labels = lifted x + noise."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, size=(B, 17 * in_F)).astype(np.float32)
    x3 = x.reshape(B, 17, in_F)
    lab = np.concatenate([x3[:, :, :2], rng.uniform(-1, 1, (B, 17, 1))], axis=2)
    lab = lab + 0.1 * rng.standard_normal(lab.shape)
    return x, lab.reshape(B, 51).astype(np.float32)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))
