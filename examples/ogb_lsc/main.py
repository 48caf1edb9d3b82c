"""RGAT on a MAG240M-like heterogeneous graph (reference: experiments/OGB-LSC/main.py).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/ogb_lsc/main.py \
        --dataset synthetic --num_papers 32768 --hidden_channels 64 --heads 4
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from dgraph_amd.experiments.ogb_lsc import cli  # noqa: E402

if __name__ == "__main__":
    cli()
