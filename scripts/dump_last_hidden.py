"""Write model.last_hidden(seqs) of the C5 shape (d 128, n 200, B 512) to an .npy file, for
comparing two builds of the library bit for bit (GR_AMD_LIB selects the build).

    GR_AMD_LIB=.../libgr_amd_x.so python scripts/dump_last_hidden.py out.npy
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
p = synth.sasrec_params(128, 200, 2, 1, 64, dev)
m = synth.sasrec_model(100_000, p, dev, seed=5)
seqs = synth.sequences(512, 200, 100_000, 5000, dev)
np.save(sys.argv[1], m.last_hidden(seqs).cpu().numpy())
