"""Row assembly behind NextRow (file_reader.go:101-108,
schema.go:171-264, data_store.go:131-203): pqgpu.rows restates getData over
decoded column chunks.  Pinned by the reference's own row vectors
(data_store_test.go: the levels and values each test asserts per leaf, and the
rows getData must return; tests/golden/rows.json), then run over whole files:
oracle-decoded columns (CPU) and GPU-decoded columns (-m gpu,
FileReader.next_row) give the same rows, and flat columns agree with pyarrow."""
import io
import json
import os

import numpy as np
import pytest

from gen import pqwrite as W
from oracle import pyoracle as O
from pqgpu import rows as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _N:
    def __init__(self, d):
        self.__dict__.update(d)


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLD, "rows.json"))), ids=lambda c: c["source"])
def test_reference_row_vectors(case):
    root = R.build_tree([_N(n) for n in case["nodes"]])
    for lf in R.leaves(root):
        c = case["leaves"][lf.leaf]
        lf.store = R.LeafStore(c["values"], np.array(c["def"], np.uint8), np.array(c["rep"], np.uint8))
    got = [R.schema_get_data(root) for _ in case["rows"]]
    assert got == case["rows"]


def _oracle_rows(pf, selected=None):
    import pqgpu  # noqa: F401
    sel = list(range(pf.num_columns)) if selected is None else selected

    def dec(rg):
        return {c: O.decode_chunk(pf.host_job(rg, c)[0]) for c in sel}
    return list(R.RowReader(pf, sel, dec))


def test_schema_nodes_of_c5():
    import pqgpu
    data, _ = W.config_c5(row_groups=(0,), rows_per_rg=500, rows_per_page=200)
    pf = pqgpu.ParquetFile(data)
    names = [(n.name.decode(), n.repetition, n.num_children, n.leaf) for n in pf.schema_nodes]
    assert names[:3] == [("lst", 1, 1, -1), ("list", 2, 1, -1), ("element", 1, 0, 0)]
    assert [n.leaf for n in pf.schema_nodes if n.num_children == 0] == list(range(pf.num_columns))


def test_oracle_rows_list_and_flat_columns():
    """C5-shaped rows (LIST<double> 3-level, optional int32, strings, ...): the
    shapes the reference's getData builds, row count = the file's rows."""
    import pqgpu
    data, _ = W.config_c5(row_groups=(0, 1), rows_per_rg=700, rows_per_page=300)
    pf = pqgpu.ParquetFile(data)
    rows = _oracle_rows(pf)
    assert len(rows) == pf.num_rows
    for r in rows[:50]:
        if "lst" in r:  # optional group: absent for a null list, {} for an empty one
            lst = r["lst"]
            assert isinstance(lst, dict)
            for e in lst.get("list", []):
                assert isinstance(e, dict) and set(e) <= {"element"}


def test_flat_rows_match_pyarrow():
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    import pqgpu
    rng = np.random.default_rng(5)
    n = 3000
    t = pa.table({"a": pa.array(rng.integers(-5, 5, n).astype(np.int32)),
                  "b": pa.array([None if rng.random() < 0.2 else float(x) for x in rng.random(n)]),
                  "s": pa.array([None if rng.random() < 0.1 else "v%d" % i for i in range(n)])})
    buf = io.BytesIO()
    pq.write_table(t, buf, data_page_size=4000, compression="snappy", row_group_size=1100)
    pf = pqgpu.ParquetFile(buf.getvalue())
    got = _oracle_rows(pf)
    exp = [{k: (v.encode() if isinstance(v, str) else v) for k, v in r.items() if v is not None}
           for r in t.to_pylist()]
    assert got == exp
    # projection: unselected columns are skipped stores (chunk_reader.go:414-420)
    got_s = _oracle_rows(pf, [pf.column_index("s")])
    assert got_s == [{"s": r["s"]} if "s" in r else {} for r in exp]


@pytest.mark.gpu
def test_gpu_next_row_matches_oracle_rows(tmp_path):
    import pqgpu
    data, _ = W.config_c5(row_groups=(0, 1, 2), rows_per_rg=1500, rows_per_page=600)
    path = tmp_path / "c5.parquet"
    path.write_bytes(data)
    pf = pqgpu.ParquetFile(data)
    exp = _oracle_rows(pf)
    fr = pqgpu.FileReader(str(path), decoder=pqgpu.GpuDecoder(0))
    try:
        got = []
        while True:
            try:
                got.append(fr.next_row())
            except EOFError:
                break
        assert len(got) == len(exp) == pf.num_rows
        assert got == exp
        # projection through FileReader: only the selected leaves appear
        fr2 = pqgpu.FileReader(str(path), "lst", "s", decoder=fr.dec)
        r0 = [fr2.next_row() for _ in range(200)]
        assert all(set(r) <= {"lst", "s"} for r in r0)
        sel = [pf.column_index("lst.list.element"), pf.column_index("s")]
        assert r0 == _oracle_rows(pf, sel)[:200]
    finally:
        fr.dec.close()
