"""Row assembly behind NextRow (file_reader.go:101-108): the restated
schema.getData (schema.go:702-712) over Column.getData / getNextData /
getFirstRDLevel (schema.go:171-264) and ColumnStore.get / getRDLevelAt
(data_store.go:131-203).

The reference walks boxed per-value ColumnStores filled by readRowGroup; here
the stores are the decoded column chunks themselves (levels + dense values, as
the GPU decode leaves them), so a Go or Python caller gets the same rows
without the per-value boxing of the decode.  Rows are dicts keyed by field
name; a REPEATED leaf yields a list of values, a REPEATED group a list of
dicts, an absent (null) field no key — the shapes of map[string]interface{},
[]T and []map[string]interface{} in the reference.  Unselected columns are
skipped stores (ColumnStore.skipped, chunk_reader.go:414-420) and never
appear."""
import numpy as np

REQUIRED, OPTIONAL, REPEATED = 0, 1, 2


class RowError(Exception):
    pass


class LeafStore:
    """One leaf column's levels and values for a row group (a ColumnStore)."""

    def __init__(self, values, def_levels, rep_levels, num_slots=None, skipped=False):
        n = num_slots if num_slots is not None else (len(def_levels) if def_levels is not None else len(values))
        self.values = values
        self.dl = def_levels if def_levels is not None else np.zeros(n, np.uint8)
        self.rl = rep_levels if rep_levels is not None else np.zeros(n, np.uint8)
        self.n = min(len(self.dl), len(self.rl))
        self.read_pos = 0
        self.vpos = 0
        self.skipped = skipped

    def rd_at(self, pos):  # getRDLevelAt data_store.go:131-148
        if pos < 0:
            pos = self.read_pos
        if pos >= self.n:
            return 0, 0, True
        return int(self.rl[pos]), int(self.dl[pos]), False

    def _next_value(self):  # getNext :150-156
        if self.vpos >= len(self.values):
            raise RowError("out of range")
        v = self.values[self.vpos]
        self.vpos += 1
        return v

    def get(self, max_d, max_r, repeated):  # get :158-203
        if self.skipped:
            return None, 0
        if self.read_pos >= self.n:
            raise RowError("out of range")
        _, dl, _ = self.rd_at(self.read_pos)
        if dl < max_d:  # a null: advance the levels, not the values
            self.read_pos += 1
            return None, dl
        v = self._next_value()
        if not repeated:
            self.read_pos += 1
            return v, max_d
        ret = [v]
        while True:
            self.read_pos += 1
            rl, _, last = self.rd_at(self.read_pos)
            if last or rl < max_r:
                return ret, max_d
            ret.append(self._next_value())


class Node:
    """A schema node (Column, schema.go): a group with children or a leaf with a store."""

    def __init__(self, name, rep, max_d, max_r, children=None, leaf=-1):
        self.name, self.rep, self.max_d, self.max_r = name, rep, max_d, max_r
        self.children = children
        self.leaf = leaf
        self.store = None


def get_data(c):  # Column.getData schema.go:235-264
    if c.children is not None:
        data, max_d = get_next_data(c)
        if c.rep != REPEATED or data is None:
            return data, max_d
        ret = [data]
        while True:
            rl, _, last = first_rd_level(c)
            if last or rl < c.max_r or rl == 0:
                return ret, max_d
            data, _ = get_next_data(c)
            ret.append(data)
    return c.store.get(c.max_d, c.max_r, c.rep == REPEATED)


def get_next_data(c):  # Column.getNextData schema.go:180-213
    ret, not_nil, max_d = {}, 0, 0
    for ch in c.children:
        data, dl = get_data(ch)
        if dl > max_d:
            max_d = dl
        if data is not None:
            ret[ch.name] = data
            not_nil += 1
        diff = 1 if ch.rep != REQUIRED else 0
        # a nil one definition level below the child's maximum: the parent is there
        if dl == ch.max_d - diff:
            not_nil += 1
    if not_nil == 0:
        return None, max_d
    return ret, c.max_d


def first_rd_level(c):  # Column.getFirstRDLevel schema.go:215-233
    if c.store is not None:
        return c.store.rd_at(-1)
    for ch in c.children:
        rl, dl, last = first_rd_level(ch)
        if last:
            return rl, dl, last
        if dl == ch.max_d:
            return rl, dl, last
    return -1, -1, False


def schema_get_data(root):  # schema.getData schema.go:702-712: a non-nil root document
    d, _ = get_data(root)
    return d if d is not None else {}


def build_tree(nodes):
    """The Column tree from depth-first (name, repetition, num_children, leaf,
    max_def, max_rep) records (pqg_file_schema_node); the root is a REQUIRED
    group at definition and repetition level 0."""
    it = iter(nodes)

    def take():
        n = next(it)
        name = n.name.decode() if isinstance(n.name, bytes) else n.name
        if n.num_children > 0:
            kids = [take() for _ in range(n.num_children)]
            return Node(name, n.repetition, n.max_def, n.max_rep, children=kids)
        return Node(name, n.repetition, n.max_def, n.max_rep, leaf=n.leaf)

    top = []
    while True:
        try:
            top.append(take())
        except StopIteration:
            break
    return Node("", REQUIRED, 0, 0, children=top)


def leaves(node):
    if node.children is None:
        return [node]
    return [x for ch in node.children for x in leaves(ch)]


def column_values(col_desc, decoded):
    """The decoded dense values of one chunk as the reference's Go values would
    compare: ints (uint32 / uint64 for unsigned columns, type_int32.go:29-33),
    floats, bools, bytes (BYTE_ARRAY, FLBA, INT96)."""
    t, flags = col_desc.physical_type, col_desc.flags
    v = decoded.values
    if decoded.offsets is not None:  # variable length
        offs = np.asarray(decoded.offsets)
        b = np.asarray(v).tobytes()
        return [b[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    raw = np.asarray(v, dtype=np.uint8)
    if t == 0:
        return [bool(x) for x in raw]
    if t == 1:
        return raw.view(np.uint32 if flags & 1 else np.int32).tolist()
    if t == 2:
        return raw.view(np.uint64 if flags & 1 else np.int64).tolist()
    if t == 4:
        return [float(x) for x in raw.view(np.float32)]
    if t == 5:
        return raw.view(np.float64).tolist()
    w = 12 if t == 3 else col_desc.type_length
    b = raw.tobytes()
    return [b[i * w:(i + 1) * w] for i in range(len(b) // w)] if w > 0 else []


class RowReader:
    """NextRow over a file's row groups (file_reader.go:93-118): the selected
    columns of each row group are decoded (by `decode_row_group(rg)` ->
    {column index: DecodedColumn}), the rest are skipped stores, and rows come
    out of schema_get_data one at a time."""

    def __init__(self, pf, selected, decode_row_group):
        self.pf = pf
        self.selected = set(selected)
        self.decode_row_group = decode_row_group
        self.root = build_tree(pf.schema_nodes)
        self.rg = 0
        self.left = 0

    def _load(self, rg):
        got = self.decode_row_group(rg)
        for lf in leaves(self.root):
            if lf.leaf not in self.selected:
                lf.store = LeafStore([], None, None, num_slots=0, skipped=True)
                continue
            d = got[lf.leaf]
            if d.status != 0:
                raise RowError("column %d of row group %d: status %d" % (lf.leaf, rg, d.status))
            lf.store = LeafStore(column_values(self.pf.columns[lf.leaf].desc, d), d.def_levels, d.rep_levels,
                                 num_slots=d.num_slots)
        self.left = self.pf.row_group_rows(rg)

    def next_row(self):
        while self.left <= 0:
            if self.rg >= self.pf.num_row_groups:
                raise EOFError
            self._load(self.rg)
            self.rg += 1
        self.left -= 1
        return schema_get_data(self.root)

    def __iter__(self):
        while True:
            try:
                yield self.next_row()
            except EOFError:
                return
