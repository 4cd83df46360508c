#!/usr/bin/env python3
"""Row-assembly known answers from the reference's data_store_test.go, written
as data to tests/golden/rows.json.

Each case is the schema the test builds (depth-first nodes: name, repetition
0/1/2, children, leaf index, maxD, maxR), the levels and values the test
asserts for every leaf column (d.data.dLevels / rLevels / values.assemble()),
and the rows getData returns (assert.Equal(t, data[i], read)).  Transcribed by
hand from the test literals (maps, []int32, []map[string]interface{} become
JSON objects and arrays); only inputs and expected outputs are kept."""
import json
import os

R, O, P = 0, 1, 2  # REQUIRED, OPTIONAL, REPEATED


def node(name, rep, children, leaf, d, r):
    return {"name": name, "repetition": rep, "num_children": children, "leaf": leaf, "max_def": d, "max_rep": r}


CASES = [
    {"source": "data_store_test.go:18-46 TestOneColumn",
     "nodes": [node("DocID", R, 0, 0, 0, 0)],
     "leaves": [{"values": [10, 20], "def": [0, 0], "rep": [0, 0]}],
     "rows": [{"DocID": 10}, {"DocID": 20}]},
    {"source": "data_store_test.go:48-74 TestOneColumnOptional",
     "nodes": [node("DocID", O, 0, 0, 1, 0)],
     "leaves": [{"values": [10], "def": [1, 0], "rep": [0, 0]}],
     "rows": [{"DocID": 10}, {}]},
    {"source": "data_store_test.go:76-102 TestOneColumnRepeated",
     "nodes": [node("DocID", P, 0, 0, 1, 1)],
     "leaves": [{"values": [10, 20], "def": [1, 1, 0], "rep": [0, 1, 0]}],
     "rows": [{"DocID": [10, 20]}, {}]},
    {"source": "data_store_test.go:104-177 TestComplexPart1",
     "nodes": [node("Name", P, 2, -1, 1, 1), node("Language", P, 2, -1, 2, 2), node("Code", R, 0, 0, 2, 2),
               node("Country", O, 0, 1, 3, 2), node("URL", O, 0, 2, 2, 1)],
     "leaves": [{"values": [1, 2, 3], "def": [2, 2, 1, 2], "rep": [0, 2, 1, 1]},
                {"values": [100, 101], "def": [3, 2, 1, 3], "rep": [0, 2, 1, 1]},
                {"values": [10, 11], "def": [2, 2, 1], "rep": [0, 1, 1]}],
     "rows": [{"Name": [{"Language": [{"Code": 1, "Country": 100}, {"Code": 2}], "URL": 10},
                        {"URL": 11},
                        {"Language": [{"Code": 3, "Country": 101}]}]}]},
    {"source": "data_store_test.go:179-225 TestComplexPart2",
     "nodes": [node("Links", O, 2, -1, 1, 0), node("Backward", P, 0, 0, 2, 1), node("Forward", P, 0, 1, 2, 1)],
     "leaves": [{"values": [10, 30], "def": [1, 2, 2], "rep": [0, 0, 1]},
                {"values": [20, 40, 60, 80], "def": [2, 2, 2, 2], "rep": [0, 1, 1, 0]}],
     "rows": [{"Links": {"Forward": [20, 40, 60]}}, {"Links": {"Backward": [10, 30], "Forward": [80]}}]},
    {"source": "data_store_test.go:227-344 TestComplex",
     "nodes": [node("DocId", R, 0, 0, 0, 0), node("Links", O, 2, -1, 1, 0), node("Backward", P, 0, 1, 2, 1),
               node("Forward", P, 0, 2, 2, 1), node("Name", P, 2, -1, 1, 1), node("Language", P, 2, -1, 2, 2),
               node("Code", R, 0, 3, 2, 2), node("Country", O, 0, 4, 3, 2), node("URL", O, 0, 5, 2, 1)],
     "leaves": [{"values": [10, 20], "def": [0, 0], "rep": [0, 0]},
                {"values": [10, 30], "def": [1, 2, 2], "rep": [0, 0, 1]},
                {"values": [20, 40, 60, 80], "def": [2, 2, 2, 2], "rep": [0, 1, 1, 0]},
                {"values": [1, 2, 3], "def": [2, 2, 1, 2, 1], "rep": [0, 2, 1, 1, 0]},
                {"values": [100, 101], "def": [3, 2, 1, 3, 1], "rep": [0, 2, 1, 1, 0]},
                {"values": [10, 11, 12], "def": [2, 2, 1, 2], "rep": [0, 1, 1, 0]}],
     "rows": [{"DocId": 10, "Links": {"Forward": [20, 40, 60]},
               "Name": [{"Language": [{"Code": 1, "Country": 100}, {"Code": 2}], "URL": 10},
                        {"URL": 11},
                        {"Language": [{"Code": 3, "Country": 101}]}]},
              {"DocId": 20, "Links": {"Backward": [10, 30], "Forward": [80]}, "Name": [{"URL": 12}]}]},
    {"source": "data_store_test.go:346-389 TestTwitterBlog",
     "nodes": [node("level1", P, 1, -1, 1, 1), node("level2", P, 0, 0, 2, 2)],
     "leaves": [{"values": list(range(1, 11)), "def": [2] * 10, "rep": [0, 2, 2, 1, 2, 2, 2, 0, 1, 2]}],
     "rows": [{"level1": [{"level2": [1, 2, 3]}, {"level2": [4, 5, 6, 7]}]},
              {"level1": [{"level2": [8]}, {"level2": [9, 10]}]}]},
    {"source": "data_store_test.go:391-427 TestEmptyParent",
     "nodes": [node("baz", O, 1, -1, 1, 0), node("list", P, 1, -1, 2, 1), node("element", R, 0, 0, 2, 1)],
     "leaves": [{"values": [], "def": [1], "rep": [0]}],
     "rows": [{"baz": {}}]},
    {"source": "data_store_test.go:429-477 TestZeroRL",
     "nodes": [node("baz", R, 1, -1, 0, 0), node("list", P, 1, -1, 1, 1), node("element", R, 1, -1, 1, 1),
               node("quux", R, 0, 0, 1, 1)],
     "leaves": [{"values": [23, 42], "def": [1, 1], "rep": [0, 1]}],
     "rows": [{"baz": {"list": [{"element": {"quux": 23}}, {"element": {"quux": 42}}]}}]},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rows.json")
    json.dump(CASES, open(out, "w"), indent=1)
    print("wrote", out, len(CASES), "cases")
