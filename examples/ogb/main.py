"""Distributed GCN on OGB node-property datasets (reference: experiments/OGB/main.py).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/ogb/main.py \
        --backend nccl --dataset products --epochs 10
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from dgraph_amd.experiments.ogb_gcn import cli  # noqa: E402

if __name__ == "__main__":
    cli()
