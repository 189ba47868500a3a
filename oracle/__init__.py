"""CPU oracle for the two hot paths — TEST INFRASTRUCTURE ONLY.

This package restates, op for op, the ATen sequence the reference runs on CPU:

* ``rq_oracle``      — ``RQVAE.get_indices`` (RQ-VAE/models/rqvae.py:67-71 → layers.py:42-43
                       → rq.py:39-56 → vq.py:63-99).
* ``sasrec_oracle``  — ``SASRec.forward`` / ``SASRec.predict`` (SASRec/model.py:49-108) with the
                       ``nn.MultiheadAttention`` slow path (torch/nn/functional.py:6576-6600).
* ``metrics_oracle`` — the rank / HR@k / NDCG@k tail of SASRec/evaluate.py:26-47.

Pinning: the restatement is checked bit-for-bit against golden vectors that
``tests/golden/make_golden.py`` produced by importing the reference itself in the
build container (see tests/test_oracle_golden.py).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / timed CPU baseline.  The product
package (``ai-education-generative-recommendation_amd/``) never imports it and has
no CPU fallback.
"""
