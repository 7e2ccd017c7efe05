#!/usr/bin/env python3
"""The staging kernel by itself (q8_stage_kernel: a batch's fp32 copy + int8 pieces), one staging at a time on an idle
GPU, for its duration without a streaming screen beside it. Run under rocprofv3 --kernel-trace --stats:
    rocprofv3 --kernel-trace --stats -d <dir> -o s -- python3 tools/stage_alone.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rag-serving-system_amd"))


def main():
    import torch
    from rag_service_amd import Index, _lib
    ix = Index(dtype="fp32", metric="cosine")
    ix.fill_synthetic(_lib.RR_SYNTH_UNIT_NORM, 1234, 125000, 1024)
    q = np.random.default_rng(3).standard_normal((16, 32, 1024)).astype(np.float32)
    dq = torch.from_numpy(q).to("cuda:0")
    torch.cuda.synchronize()
    for i in range(300):
        ix.set_queries_device(dq[i % 16].data_ptr(), 32, 1024)
        ix.synchronize()
    ix.close()
    print("ok")


if __name__ == "__main__":
    main()
