"""The reference's kmer data directory on disk.

    <dir>/kmer.table.mem_map   header {u64 num_sigs, u64 entry_size=24, i64 version=1}
                               + num_sigs 24-byte buckets (kmer_image.h:11-23,
                               written by save_kmer_hash_table, kguts.cc:224-234)
    <dir>/function.index       "%d\\t<function>\\n", dense and in order (kguts.cc:544-575)
    <dir>/otu.index            same format
"""
from __future__ import annotations

import os

import numpy as np

from .abi import SIG_DTYPE

HEADER = np.dtype([("num_sigs", "<u8"), ("entry_size", "<u8"), ("version", "<i8")])


def write_image(data_dir: str, table: np.ndarray) -> str:
    os.makedirs(data_dir, exist_ok=True)
    table = np.ascontiguousarray(table)
    assert table.dtype.itemsize == 24
    hdr = np.array([(len(table), 24, 1)], dtype=HEADER)
    path = os.path.join(data_dir, "kmer.table.mem_map")
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(table.tobytes())
    return path


def read_image(data_dir: str) -> np.ndarray:
    path = os.path.join(data_dir, "kmer.table.mem_map")
    hdr = np.fromfile(path, dtype=HEADER, count=1)[0]
    return np.fromfile(path, dtype=SIG_DTYPE, offset=HEADER.itemsize, count=int(hdr["num_sigs"]))


def write_index(path: str, names: list[str]) -> None:
    with open(path, "w") as f:
        for i, n in enumerate(names):
            f.write(f"{i}\t{n}\n")


def write_data_dir(data_dir: str, table: np.ndarray, functions: list[str],
                   otus: list[str] | None = None) -> str:
    write_image(data_dir, table)
    write_index(os.path.join(data_dir, "function.index"), functions)
    write_index(os.path.join(data_dir, "otu.index"), otus if otus is not None else ["otu0"])
    return data_dir
