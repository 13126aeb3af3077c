"""Fixed workload for rocprofv3: 4 batches of the split-phase scrypt ROMix (write launch, lookup launch)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from otedama_amd.ops.search import ScryptSearch  # noqa: E402

s = ScryptSearch("cuda:0", kernel="split")
p = s.prepare(bytes(range(76)) + bytes(4), bytes(32))
for i in range(4):
    s.launch(p, i * s.batch)
torch.cuda.synchronize()
print("done")
