"""Host handling of timestamp strings outside the engine's canonical domain
(the server's request path; evolu_amd/server.py).

The reference server stores a message's timestamp as sent and XORs
insertIntoMerkleTree(timestampFromString(raw)) into the owner's tree
(apps/server/src/index.ts:151-159).  timestampFromString
(packages/evolu/src/timestamp.ts:50-55) splits at '-', Date.parse's the date
part, parseInt's the counter, keeps the node; the tree hashes
timestampToString of the result (timestamp.ts:43-48), whose toISOString
throws a RangeError on an invalid date -- the whole request then rolls back
and the server answers 500 (index.ts:166-169).

`classify(raw)` restates that for the ISO-shaped strings V8 parses with its
ES5 ISO parser (fixed-width fields; it rolls days 29-31 over into the next
month and takes hour 24 at :00:00.000; 't' and 'z' in either case), pinned by
node-generated vectors (tests/golden/js_lenient.json):
  ("ok", canonical)   -- what the tree sees, inside the engine's native domain
  ("range_error", None) -- Date.parse is NaN: the request fails (500)
  ("unsupported", None) -- a form this host path does not model
"""
from __future__ import annotations

import re
from typing import Optional, Tuple

_ISO = re.compile(r"^(\d{4})-(\d{2})-(\d{2})[Tt](\d{2}):(\d{2}):(\d{2})\.(\d{3})[Zz]$")
_HEX4 = re.compile(r"^[0-9a-fA-F]{4}$")
_NODE = re.compile(r"^[0-9a-fA-F]{16}$")
MS_PER_DAY = 86400000
NATIVE_END = 2 ** 31 * 60000  # the engine's native domain: 1970 <= t < 2^31 minutes


def _days_from_civil(y: int, m: int, d: int) -> int:
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def _civil_from_days(z: int):
    z += 719468
    era = (z if z >= 0 else z - 146096) // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + 3 if mp < 10 else mp - 9
    return y + (m <= 2), m, d


def date_parse(s: str) -> Optional[int]:
    """V8's Date.parse on the ISO shape above -> millis, None for NaN.
    Raises ValueError for a string of another shape (not modelled)."""
    mt = _ISO.match(s)
    if not mt:
        raise ValueError("not an ISO-shaped date: %r" % s)
    y, mo, d, hh, mi, ss, ms = (int(mt.group(k)) for k in range(1, 8))
    if not (1 <= mo <= 12 and 1 <= d <= 31 and hh <= 24 and mi <= 59 and ss <= 59):
        return None
    if hh == 24 and (mi or ss or ms):
        return None
    days = _days_from_civil(y, mo, 1) + d - 1  # MakeDay: a day past the month's end rolls over
    return days * MS_PER_DAY + ((hh * 60 + mi) * 60 + ss) * 1000 + ms


def to_string(millis: int, counter: int, node: str) -> Optional[str]:
    """timestamp.ts:43-48 for a 4-digit year (None: toISOString would give
    an extended +YYYYYY year, outside the 46-byte form)."""
    days, rem = divmod(millis, MS_PER_DAY)
    y, m, d = _civil_from_days(days)
    if not 0 <= y <= 9999 or not 0 <= counter <= 0xFFFF:
        return None
    hh, rem = divmod(rem, 3600000)
    mi, rem = divmod(rem, 60000)
    ss, ms = divmod(rem, 1000)
    return "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ-%04X-%s" % (y, m, d, hh, mi, ss, ms, counter, node)


def classify(raw: str) -> Tuple[str, Optional[str]]:
    a = raw.split("-")
    if len(a) != 5 or not _HEX4.match(a[3]) or not _NODE.match(a[4]):
        return "unsupported", None
    try:
        millis = date_parse("-".join(a[:3]))
    except ValueError:
        return "unsupported", None
    if millis is None:
        return "range_error", None
    canon = to_string(millis, int(a[3], 16), a[4])
    if canon is None or not 0 <= millis < NATIVE_END:
        return "unsupported", None
    return "ok", canon
