"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the SUTA adapt loop.

Nothing in the product path (the `suta_amd` package, `libsuta.so`) imports,
links or executes anything under `oracle/`.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use it, and only
as the checker / the timed CPU baseline.

Contents
- `w2v2_cpu.py`   : PyTorch-CPU functional restatement of Wav2Vec2ForCTC forward
                    (HF transformers 5.15.0 modeling_wav2vec2.py), the SUTA loss
                    (reference main.py:26-60, 181-203), `collect_params`
                    multiplicity (main.py:62-103) and single-tensor AdamW with
                    duplicate-entry sub-steps (torch/optim/adam.py:347-548).
- `suta_loss_np.py`: float64 NumPy closed form of the fused entropy+MCC
                    loss-and-gradient.

Pinning: both restatements are checked against golden vectors produced by
running the reference's own `main.py` functions (imported with a `jiwer` stub)
on seeded inputs; see `tests/golden/make_golden.py` and
`tests/test_oracle_golden.py`.
"""
