"""CPU oracle for the Evolu CRDT sync hot path -- TEST INFRASTRUCTURE ONLY.

This module is a line-by-line restatement of the reference's hot-path
functions in plain Python.  It is the *checker* for the HIP engine: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it.  The product path (``evolu_amd``) never imports it and
fails loudly when the HIP library is missing.

Parity pinning: the reference is TypeScript with no installed toolchain
(no ``tsc``, no ``node_modules``), so it cannot run here.  The restatement
is pinned instead by every golden value the reference's own tests hold
(``packages/evolu/test/__snapshots__/*.snap``, see ``tests/golden/``) and
by an independent murmur3 (Debian ``imurmurhash`` 0.1.4 under node 12,
``oracle/js/gen_murmur_vectors.js``).  ``applyMessages`` and the server's
``addMessages``/``getMessages`` have no reference tests: they are pinned by
running the reference's SQL statements verbatim in ``sqlite3``.

JS semantics emulated (each cited where used): IEEE-double arithmetic,
ToInt32 on ``^`` and ``|0``, ``Number#toString(3)``, ``parseInt(s, 3)``,
``Date#toISOString``, JSON.stringify key order of ``MerkleTree``.
"""
from __future__ import annotations

import json
import re
import sqlite3
import struct
from typing import Dict, List, Optional, Sequence, Tuple

# --------------------------------------------------------------------------
# JS number helpers
# --------------------------------------------------------------------------


def to_int32(x) -> int:
    """ECMAScript ToInt32 (used by ``^`` and ``|0``)."""
    if x is None:  # ToInt32(undefined) == ToInt32(NaN) == 0
        return 0
    if isinstance(x, float):
        if x != x or x in (float("inf"), float("-inf")):
            return 0
        x = int(x)  # truncation toward zero
    x &= 0xFFFFFFFF
    return x - 0x100000000 if x & 0x80000000 else x


def js_to_string_radix(n: int, radix: int) -> str:
    """``Number.prototype.toString(radix)`` for an integral number."""
    if n == 0:
        return "0"
    digits = "0123456789abcdefghijklmnopqrstuvwxyz"
    neg = n < 0
    n = -n if neg else n
    out = []
    while n:
        n, r = divmod(n, radix)
        out.append(digits[r])
    return ("-" if neg else "") + "".join(reversed(out))


# --------------------------------------------------------------------------
# murmurhash@2.0.1 (npm) == MurmurHash3_x86_32, seed 0, over UTF-8 bytes.
# Reference call site: packages/evolu/src/timestamp.ts:6,87-88.
# --------------------------------------------------------------------------

_C1, _C2 = 0xCC9E2D51, 0x1B873593
_M32 = 0xFFFFFFFF


def _rotl32(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & _M32


def murmur3_32(data: bytes, seed: int = 0) -> int:
    """MurmurHash3_x86_32 -> uint32 (the npm package returns ``h >>> 0``)."""
    h = seed & _M32
    n = len(data)
    nblocks = n // 4
    for i in range(nblocks):
        (k,) = struct.unpack_from("<I", data, 4 * i)
        k = (k * _C1) & _M32
        k = _rotl32(k, 15)
        k = (k * _C2) & _M32
        h ^= k
        h = _rotl32(h, 13)
        h = (h * 5 + 0xE6546B64) & _M32
    tail = data[4 * nblocks:]
    k = 0
    if len(tail) >= 3:
        k ^= tail[2] << 16
    if len(tail) >= 2:
        k ^= tail[1] << 8
    if len(tail) >= 1:
        k ^= tail[0]
        k = (k * _C1) & _M32
        k = _rotl32(k, 15)
        k = (k * _C2) & _M32
        h ^= k
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & _M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & _M32
    h ^= h >> 16
    return h


# --------------------------------------------------------------------------
# Dates: Date#toISOString and the strict (canonical) subset of Date.parse.
# --------------------------------------------------------------------------

MS_PER_DAY = 86400000
MAX_COUNTER = 65535  # types.ts:54


def _days_from_civil(y: int, m: int, d: int) -> int:
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def _civil_from_days(z: int) -> Tuple[int, int, int]:
    z += 719468
    era = (z if z >= 0 else z - 146096) // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + (3 if mp < 10 else -9)
    return y + (m <= 2), m, d


def _days_in_month(y: int, m: int) -> int:
    if m == 2:
        leap = (y % 4 == 0 and y % 100 != 0) or y % 400 == 0
        return 29 if leap else 28
    return 31 if m in (1, 3, 5, 7, 8, 10, 12) else 30


def iso_string(millis: int) -> str:
    """``new Date(millis).toISOString()`` (timestamp.ts:45)."""
    if not (-8.64e15 <= millis <= 8.64e15):
        raise ValueError("RangeError: Invalid time value")
    days, ms = divmod(int(millis), MS_PER_DAY)
    y, m, d = _civil_from_days(days)
    hh, rem = divmod(ms, 3600000)
    mm, rem = divmod(rem, 60000)
    ss, sss = divmod(rem, 1000)
    if 0 <= y <= 9999:
        ys = "%04d" % y
    else:
        ys = ("+" if y > 0 else "-") + "%06d" % abs(y)
    return "%s-%02d-%02dT%02d:%02d:%02d.%03dZ" % (ys, m, d, hh, mm, ss, sss)


_CANON = re.compile(
    r"^(\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2}):(\d{2})\.(\d{3})Z-([0-9A-F]{4})-([0-9a-fA-F]{16})$"
)


class NonCanonical(ValueError):
    """A timestamp string outside the engine's bit-exact native domain."""


def parse_canonical(s: str) -> Tuple[int, int, str]:
    """Strict parse of a timestamp string S with S == toString(fromString(S)).

    Follows timestamp.ts:50-55 (``split('-')``, ``Date.parse`` of the first
    three parts, ``parseInt(a[3], 16)``, ``a[4]``) restricted to strings that
    round-trip through timestamp.ts:43-48 unchanged.  Anything else (V8's
    lenient date forms, lower-case counter hex, extended years) raises
    ``NonCanonical``.
    """
    mt = _CANON.match(s)
    if not mt:
        raise NonCanonical(s)
    y, mo, d, hh, mi, ss, sss = (int(mt.group(i)) for i in range(1, 8))
    if not (1 <= mo <= 12 and 1 <= d <= _days_in_month(y, mo)):
        raise NonCanonical(s)
    if hh > 23 or mi > 59 or ss > 59:
        raise NonCanonical(s)
    millis = ((_days_from_civil(y, mo, d) * 24 + hh) * 60 + mi) * 60000 + ss * 1000 + sss
    return millis, int(mt.group(8), 16), mt.group(9)


# --------------------------------------------------------------------------
# timestamp.ts
# --------------------------------------------------------------------------


def timestamp_to_string(millis: int, counter: int, node: str) -> str:
    """timestamp.ts:43-48."""
    return "-".join([iso_string(millis), ("%x" % counter).upper().rjust(4, "0"), node])


def timestamp_from_string(s: str) -> Tuple[int, int, str]:
    """timestamp.ts:50-55, canonical domain (see ``parse_canonical``)."""
    return parse_canonical(s)


def timestamp_to_hash(millis: int, counter: int, node: str) -> int:
    """timestamp.ts:87-88 -> uint32."""
    return murmur3_32(timestamp_to_string(millis, counter, node).encode("utf-8"))


_ISO_JS = re.compile(r"^(\d{4})-(\d{2})-(\d{2})[Tt](\d{2}):(\d{2}):(\d{2})\.(\d{3})[Zz]$")
_PARSE_INT_16 = re.compile(r"^\s*([+-]?)(?:0[xX])?([0-9a-fA-F]+)")


def date_parse_js(s: str) -> Optional[int]:
    """V8 ``Date.parse`` of an ISO-shaped date string (its ES5 ISO parser:
    fixed-width fields, a day up to 31 rolls over past the month's end (MakeDay),
    hour 24 only at :00:00.000, 't'/'z' in either case) -> millis, None for
    NaN.  Other shapes raise NonCanonical (V8's legacy parser: not modelled).
    Pinned by node: tests/golden/js_lenient.json (oracle/js/gen_lenient.js)."""
    mt = _ISO_JS.match(s)
    if not mt:
        raise NonCanonical(s)
    y, mo, d, hh, mi, ss, ms = (int(mt.group(i)) for i in range(1, 8))
    if not (1 <= mo <= 12 and 1 <= d <= 31 and hh <= 24 and mi <= 59 and ss <= 59):
        return None
    if hh == 24 and (mi or ss or ms):
        return None
    return (_days_from_civil(y, mo, 1) + d - 1) * MS_PER_DAY + ((hh * 60 + mi) * 60 + ss) * 1000 + ms


def timestamp_from_string_js(s: str) -> Tuple[Optional[int], int, str]:
    """timestamp.ts:50-55 as written: ``a = s.split("-")``; millis =
    ``Date.parse(a.slice(0, 3).join("-"))`` (None for NaN), counter =
    ``parseInt(a[3], 16)``, node = ``a[4]``.  Canonical strings take
    parse_canonical; a counter or node JS would turn into NaN / undefined is
    not modelled (NonCanonical)."""
    try:
        return parse_canonical(s)
    except NonCanonical:
        pass
    a = s.split("-")
    if len(a) < 5:
        raise NonCanonical(s)
    mt = _PARSE_INT_16.match(a[3])
    if not mt:
        raise NonCanonical(s)
    counter = int(mt.group(2), 16) * (-1 if mt.group(1) == "-" else 1)
    return date_parse_js("-".join(a[:3])), counter, a[4]


def create_sync_timestamp(millis: int = 0) -> Tuple[int, int, str]:
    """timestamp.ts:35-41."""
    return (millis, 0, "0000000000000000")


class TimestampError(Exception):
    def __init__(self, kind: str, **kw):
        super().__init__(kind)
        self.kind = kind
        self.info = kw


def send_timestamp(ts: Tuple[int, int, str], now: int, max_drift: int = 60000):
    """timestamp.ts:97-123."""
    millis, counter, node = ts
    nxt = max(millis, now)
    if nxt - now > max_drift:
        raise TimestampError("TimestampDriftError", next=nxt, now=now)
    if nxt == millis:
        if counter >= MAX_COUNTER:
            raise TimestampError("TimestampCounterOverflowError")
        c = counter + 1
    else:
        c = 0
    return (nxt, c, node)


def receive_timestamp(local, remote, now: int, max_drift: int = 60000):
    """timestamp.ts:125-165."""
    nxt = max(local[0], remote[0], now)
    if nxt - now > max_drift:
        raise TimestampError("TimestampDriftError", next=nxt, now=now)
    if local[2] == remote[2]:
        raise TimestampError("TimestampDuplicateNodeError", node=local[2])
    if nxt == local[0] and nxt == remote[0]:
        base = max(local[1], remote[1])
    elif nxt == local[0]:
        base = local[1]
    elif nxt == remote[0]:
        base = remote[1]
    else:
        return (nxt, 0, local[2])
    if base >= MAX_COUNTER:
        raise TimestampError("TimestampCounterOverflowError")
    return (nxt, base + 1, local[2])


# --------------------------------------------------------------------------
# merkleTree.ts -- literal persistent trie (dicts with keys "0","1","2","hash")
# --------------------------------------------------------------------------


def minute_key(millis: int) -> str:
    """merkleTree.ts:33: ``Number((millis / 1000 / 60) | 0).toString(3)``."""
    return js_to_string_radix(to_int32(float(millis) / 1000.0 / 60.0), 3)


def _insert_key(tree: dict, key: str, h: int) -> dict:
    """merkleTree.ts:8-29."""
    if len(key) == 0:
        return tree
    c = key[0]
    n = tree.get(c) or {}
    child = dict(n)
    child.update(_insert_key(n, key[1:], h))
    child["hash"] = to_int32(to_int32(n.get("hash")) ^ to_int32(h))
    out = dict(tree)
    out[c] = child
    return out


def insert_into_merkle_tree(tree: dict, ts: Tuple[int, int, str]) -> dict:
    """merkleTree.ts:31-50."""
    key = minute_key(ts[0])
    h = timestamp_to_hash(*ts)
    root = dict(tree)
    root["hash"] = to_int32(to_int32(tree.get("hash")) ^ to_int32(h))
    return _insert_key(root, key, h)


def _get_keys(tree: dict) -> List[str]:
    """merkleTree.ts:52-53 (JS orders integer-like keys first)."""
    return [k for k in tree.keys() if k != "hash"]


class RangeErrorJS(Exception):
    """JS RangeError (``"0".repeat(-1)`` in keyToTimestamp)."""


def key_to_timestamp(key: str) -> int:
    """merkleTree.ts:55-61."""
    if len(key) > 16:
        raise RangeErrorJS("Invalid count value: %d" % (16 - len(key)))
    full = key + "0" * (16 - len(key))
    return int(full, 3) * 1000 * 60


def diff_merkle_trees(t1: dict, t2: dict) -> Optional[int]:
    """merkleTree.ts:63-91.  Returns None (option.none) or millis."""
    if t1.get("hash") == t2.get("hash"):
        return None
    n1, n2, k = t1, t2, ""
    while True:
        keys = sorted(set(_get_keys(n1)) | set(_get_keys(n2)))
        diffkey = None
        for key in keys:
            a = n1.get(key) or {}
            b = n2.get(key) or {}
            if a.get("hash") != b.get("hash"):
                diffkey = key
                break
        if diffkey is None:
            return key_to_timestamp(k)
        k += diffkey
        n1 = n1.get(diffkey) or {}
        n2 = n2.get(diffkey) or {}


def merkle_tree_to_string(tree: dict) -> str:
    """types.ts:80-81 ``JSON.stringify`` (integer keys ascending, then "hash")."""

    def emit(t: dict) -> str:
        parts = []
        for k in ("0", "1", "2"):
            if k in t:
                parts.append('"%s":%s' % (k, emit(t[k])))
        if "hash" in t:
            parts.append('"hash":%d' % t["hash"])
        return "{" + ",".join(parts) + "}"

    return emit(tree)


def merkle_tree_from_string(s: str) -> dict:
    """types.ts:83-84."""
    return json.loads(s)


# --------------------------------------------------------------------------
# Leaf-map view of a trie (the engine's representation), for comparisons.
# A leaf is (key string, xor) for every key that received >= 1 insert.
# --------------------------------------------------------------------------


def tree_from_leaves(leaves: Dict[str, int]) -> dict:
    """Builds the literal trie whose inserts terminate at ``leaves``."""
    root: dict = {}
    if not leaves:
        return root
    h_all = 0
    for key, x in leaves.items():
        h_all ^= x
        node = root
        for c in key:
            node = node.setdefault(c, {})
            node["hash"] = to_int32(node.get("hash", 0) ^ x)
    root["hash"] = to_int32(h_all)
    return root


# --------------------------------------------------------------------------
# applyMessages.ts -- verbatim SQL in sqlite3, control flow restated.
# --------------------------------------------------------------------------

_SQL_SELECT_MOST_RECENT = """
          SELECT "timestamp" FROM "__message"
          WHERE "table" = ? AND
                "row" = ? AND
                "column" = ?
          ORDER BY "timestamp" DESC LIMIT 1
        """  # applyMessages.ts:34-40

_SQL_INSERT_MESSAGE = """
          INSERT INTO "__message" (
            "timestamp", "table", "row", "column", "value"
          ) VALUES (?, ?, ?, ?, ?) ON CONFLICT DO NOTHING
        """  # applyMessages.ts:41-45

_SQL_CLIENT_SCHEMA = """
          CREATE TABLE __message (
            "timestamp" BLOB PRIMARY KEY,
            "table" BLOB,
            "row" BLOB,
            "column" BLOB,
            "value" BLOB
          );

          CREATE INDEX index__message ON __message (
            "table",
            "row",
            "column",
            "timestamp"
          );
"""  # initDbModel.ts:43-56


class ClientDb:
    """A client's SQLite state (``__message`` + user tables), in memory."""

    def __init__(self):
        self.conn = sqlite3.connect(":memory:")
        self.conn.executescript(_SQL_CLIENT_SCHEMA)
        self.tables: Dict[str, set] = {}

    def ensure_table(self, table: str, column: str):
        """updateDbSchema.ts:61-78 (``"id" TEXT PRIMARY KEY`` + BLOB columns)."""
        cols = self.tables.get(table)
        if cols is None:
            self.conn.execute('CREATE TABLE "%s" ("id" TEXT PRIMARY KEY, "%s" BLOB)' % (table, column))
            self.tables[table] = {column}
        elif column not in cols:
            self.conn.execute('ALTER TABLE "%s" ADD COLUMN "%s" BLOB' % (table, column))
            cols.add(column)

    def cell_max(self, table, row, column) -> Optional[str]:
        r = self.conn.execute(_SQL_SELECT_MOST_RECENT, (table, row, column)).fetchone()
        return None if r is None else r[0]

    def messages(self):
        return self.conn.execute('SELECT * FROM "__message" ORDER BY "timestamp"').fetchall()

    def table_rows(self, table):
        return self.conn.execute('SELECT * FROM "%s" ORDER BY "id"' % table).fetchall()


def apply_messages(db: ClientDb, tree: dict, messages: Sequence[dict], decisions: Optional[list] = None) -> dict:
    """applyMessages.ts:26-131.

    ``messages`` are dicts {timestamp, table, row, column, value}.  Returns
    the new MerkleTree.  When ``decisions`` is a list, appends per message a
    tuple (ups, xor, ins) -- the upsert taken (:93), the Merkle XOR taken
    (:105,:114-119) and whether the INSERT changed a row (:107-113).
    """
    cur = db.conn.cursor()
    for m in messages:
        r = cur.execute(_SQL_SELECT_MOST_RECENT, (m["table"], m["row"], m["column"])).fetchone()
        t = None if r is None else r[0]
        ups = t is None or t < m["timestamp"]  # :93, JS string '<' == code-unit order
        if ups:
            db.ensure_table(m["table"], m["column"])
            cur.execute(
                'INSERT INTO "%s" ("id", "%s") VALUES (?, ?) ON CONFLICT DO UPDATE SET "%s" = ?'
                % (m["table"], m["column"], m["column"]),
                (m["row"], m["value"], m["value"]),
            )  # :94-101
        xor = t is None or t != m["timestamp"]  # :105
        ins = False
        if xor:
            cur.execute(_SQL_INSERT_MESSAGE, (m["timestamp"], m["table"], m["row"], m["column"], m["value"]))
            ins = cur.rowcount == 1
            tree = insert_into_merkle_tree(tree, timestamp_from_string(m["timestamp"]))  # :114-119
        if decisions is not None:
            decisions.append((ups, xor, ins))
    return tree


# --------------------------------------------------------------------------
# apps/server/src/index.ts -- verbatim SQL in sqlite3.
# --------------------------------------------------------------------------

_SQL_SERVER_SCHEMA = """
      CREATE TABLE IF NOT EXISTS "message" (
        "timestamp" TEXT,
        "userId" TEXT,
        "content" BLOB,
        PRIMARY KEY(timestamp, userId)
      );
      CREATE TABLE IF NOT EXISTS "merkleTree" (
        "userId" TEXT PRIMARY KEY,
        "merkleTree" TEXT
      );
"""  # index.ts:64-75

_SQL_SELECT_TREE = 'SELECT "merkleTree" FROM "merkleTree" WHERE "userId" = ?'  # :82-84
_SQL_INSERT_OR_IGNORE = """
        INSERT OR IGNORE INTO "message" (
          "timestamp", "userId", "content"
        ) VALUES (?, ?, ?) ON CONFLICT DO NOTHING
      """  # :86-90
_SQL_SAVE_TREE = """
        INSERT OR REPLACE INTO "merkleTree" (
          "userId", "merkleTree"
        ) VALUES (?, ?)
      """  # :92-96
_SQL_SELECT_MESSAGES = """
        SELECT "timestamp", "content" FROM "message"
        WHERE "userId" = ? AND "timestamp" > ? AND "timestamp" NOT LIKE '%' || ?
        ORDER BY "timestamp"
      """  # :98-102


class ServerDb:
    def __init__(self):
        self.conn = sqlite3.connect(":memory:", isolation_level=None)
        self.conn.executescript(_SQL_SERVER_SCHEMA)

    def get_merkle_tree(self, user_id: str) -> dict:
        """index.ts:121-136."""
        r = self.conn.execute(_SQL_SELECT_TREE, (user_id,)).fetchone()
        return merkle_tree_from_string(r[0]) if r else {}

    def add_messages(self, tree: dict, user_id: str, messages: Sequence[Tuple[str, bytes]], inserted: Optional[list] = None) -> dict:
        """index.ts:138-171.  ``messages`` = [(timestamp, content)]."""
        if len(messages) == 0:
            return tree
        cur = self.conn.cursor()
        cur.execute("BEGIN")
        try:
            for ts, content in messages:
                cur.execute(_SQL_INSERT_OR_IGNORE, (ts, user_id, content))
                took = cur.rowcount == 1
                if inserted is not None:
                    inserted.append(took)
                if took:
                    # the raw string is stored; the tree sees timestampFromString(raw)
                    # (lenient), whose toISOString throws on an invalid date
                    t = timestamp_from_string_js(ts)
                    if t[0] is None:
                        raise RangeErrorJS("Invalid time value")
                    tree = insert_into_merkle_tree(tree, t)
            cur.execute(_SQL_SAVE_TREE, (user_id, merkle_tree_to_string(tree)))
            cur.execute("COMMIT")
        except Exception:
            cur.execute("ROLLBACK")
            raise
        return tree

    def get_messages(self, tree: dict, client_tree: dict, user_id: str, node_id: str):
        """index.ts:173-202 -> (diff or None, [(timestamp, content)])."""
        diff = diff_merkle_trees(tree, client_tree)
        if diff is None:
            return None, []
        since = timestamp_to_string(*create_sync_timestamp(diff))
        rows = self.conn.execute(_SQL_SELECT_MESSAGES, (user_id, since, node_id)).fetchall()
        return diff, rows

    def sync(self, user_id: str, node_id: str, client_tree_json: str, messages):
        """index.ts:204-216."""
        tree = self.get_merkle_tree(user_id)
        tree = self.add_messages(tree, user_id, messages)
        diff, rows = self.get_messages(tree, merkle_tree_from_string(client_tree_json), user_id, node_id)
        return tree, diff, rows
