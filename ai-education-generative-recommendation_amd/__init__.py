"""gr_amd — MI355X (gfx950) implementation of the two data-parallel hot paths of
CatchMan1/AI-education-generative-recommendation:

* RQ-VAE residual-quantization encode  (``RQVAE.get_indices``)  -> ``gr_amd.rqvae``
* SASRec forward / full-catalog scoring (``SASRec.predict``)     -> ``gr_amd.sasrec``

The directory name is not a Python identifier; the repository root's ``gr_amd.py`` registers it
under the import name ``gr_amd``.  Kernels live in ``csrc/`` behind the C ABI of include/gr_amd.h
and are loaded from ``lib/libgr_amd.so`` (built by ``build.py``); there is no CPU fallback.
"""
from . import ops  # noqa: F401
from ._lib import LIB_PATH, lib  # noqa: F401
from .rqvae import RQVAE  # noqa: F401
from .sasrec import SASRec  # noqa: F401

__all__ = ["RQVAE", "SASRec", "ops", "lib", "LIB_PATH"]
