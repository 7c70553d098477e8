"""Synthetic utterances for benches and parity tests.

Utterance i of length N: `np.random.default_rng(20260415 + i).standard_normal(N) * 0.05`,
float32, then the HF processor's normalisation (feature_extraction_wav2vec2.py:78-97).
"""
import numpy as np

SEED = 20260415


def raw_wave(n: int, i: int = 0, seed: int = SEED) -> np.ndarray:
    return np.random.default_rng(seed + i).standard_normal(n, dtype=np.float32) * np.float32(0.05)


def normalize(x: np.ndarray) -> np.ndarray:
    """(x - mean) / sqrt(var + 1e-7) in float32, as Wav2Vec2FeatureExtractor.zero_mean_unit_var_norm."""
    x = np.asarray(x, dtype=np.float32)
    return ((x - x.mean()) / np.sqrt(x.var() + 1e-7)).astype(np.float32)


def wave(n: int, i: int = 0, seed: int = SEED) -> np.ndarray:
    return normalize(raw_wave(n, i, seed))


def batch(n: int, count: int, start: int = 0) -> np.ndarray:
    return np.stack([wave(n, start + i) for i in range(count)])
