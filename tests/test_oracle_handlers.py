"""CPU checks of the oracle's handler restatements (oracle/handlers_oracle.cpp)
on hand-worked cases read off the reference (no GPU)."""
import numpy as np


def test_kmap_append_keeps_duplicates_set_keeps_first(oracle_lib):
    """add_mapping appends (kmer.cc:173-210); add_fam_mapping skips ids already
    in the list (fam_map_insert, kmer.cc:214-227)."""
    a, s = oracle_lib.Kmap(0), oracle_lib.Kmap(1)
    k = [10, 10, 11, 10, 10, 11]
    v = [3, 1, 4, 3, 2, 4]
    a.add(k, v)
    s.add(k, v)
    assert a.lookup(10).tolist() == [3, 1, 3, 2] and a.lookup(11).tolist() == [4, 4]
    assert s.lookup(10).tolist() == [3, 1, 2] and s.lookup(11).tolist() == [4]
    assert a.lookup(12).tolist() == [] and a.num_kmers == 2


def test_matrix_counts_only_ids_seen_earlier_in_the_request(oracle_lib):
    """matrix_request.cc:89-95,143-150: the id joins matrix_proteins_ before its
    hits are scanned; partners must already be in matrix_proteins_ and differ
    from the sequence's own id; duplicates in a k-mer list count twice."""
    km = oracle_lib.Kmap(0)
    # /add: protein 1 has k-mers A,B; protein 2 has A,A(twice),C; protein 3 has B
    A, B, C = 100, 200, 300
    km.add([A, B, A, A, C, B], [1, 1, 2, 2, 2, 3])
    mx = oracle_lib.Matrix()
    # request: 2 (len 10) then 1 (len 20) then 3 (len 30) then 2 again (len 40)
    off = np.array([0, 2, 4, 5, 6], np.uint64)
    kmers = np.array([A, C, A, B, B, A], np.uint64)
    mx.add(km, [2, 1, 3, 2], [10, 20, 30, 40], off, kmers)
    id1, id2, cnt, score = mx.pairs()
    got = {(int(a), int(b)): int(c) for a, b, c in zip(id1, id2, cnt)}
    # seq 0 (id 2): A -> [1,2,2]: 1 not seen yet; C -> [2]: self.  Nothing.
    # seq 1 (id 1): A -> 1 self, 2 seen twice -> (1,2)+=2; B -> [1,3]: 3 unseen
    # seq 2 (id 3): B -> [1,3]: (3,1)+=1
    # seq 3 (id 2): A -> [1,2,2]: (2,1)+=1
    assert got == {(1, 2): 2, (2, 1): 1, (3, 1): 1}
    assert list(zip(id1.tolist(), id2.tolist())) == [(1, 2), (2, 1), (3, 1)]  # std::map order
    # score uses the last length recorded for each id (matrix_proteins_[eid] = size)
    assert score[0] == np.float32(2) / np.float32(20 + 40)
