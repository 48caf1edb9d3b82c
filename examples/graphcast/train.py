"""GraphCast on synthetic ERA5-shaped data (reference: experiments/GraphCast/train_graphcast.py).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/graphcast/train.py \
        --backend nccl --procs_per_graph 4 --iters 100 --dtype bf16
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from dgraph_amd.experiments.graphcast import cli  # noqa: E402

if __name__ == "__main__":
    cli()
