"""Split helpers (DGraph/utils/data_splitting.py)."""


def largest_split(global_size: int, world_size: int) -> int:
    """Size of the largest of ``world_size`` near-equal contiguous splits (ceil div)."""
    return (global_size + world_size - 1) // world_size


def split_per_rank(global_size: int, world_size: int, rank: int) -> tuple:
    """[start, end) of ``rank``'s near-equal contiguous split."""
    base, rem = divmod(global_size, world_size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)
