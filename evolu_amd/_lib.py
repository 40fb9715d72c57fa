"""ctypes binding of the C ABI in include/evm.h (libevm.so, built in-tree).

There is no fallback: if the HIP library is missing or cannot be loaded the
import of anything that computes raises, by design.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libevm.so")

EVM_OK = 0
EVM_EINVAL = 1
EVM_ENONCANON = 2
EVM_ECOLLISION = 3
EVM_ERANGE = 4
EVM_ETREE = 5
EVM_EDEVICE = 6
EVM_ENOMEM = 7
EVM_ECAPACITY = 8
EVM_EDIST = 9
EVM_ESTATE = 10
EVM_EROUNDS = 11
EVM_EHANDOVER = 12
SYNC_HOST = 0
SYNC_DEVICE = 1
DIST_ID_BYTES = 128

META_CASEMASK = 0x0000FFFF
META_VALID = 0x00010000
META_NONCANON = 0x00020000
META_RANGE = 0x00040000

MSG_UPS = 0x01
MSG_XOR = 0x02
MSG_INS = 0x04
ROUTE_NO_SRC = 1  # evm_dist_route_ex: no source indexes wanted (24-B records when aux is absent)
ROUTE_KEEP_INPUT = 2  # ... and the caller keeps ts until the last take / ingest (own rows never copied)
MSG_BAD = 0x80

OPT_CLIENT_PATH = 1
OPT_SERVER_PATH = 2
OPT_OVERLAP = 3
OPT_RADIX = 4
OPT_DIFF_GRID = 6
OPT_SELECT_PATH = 7

PB_SYNC_REQUEST = 1
PB_SYNC_RESPONSE = 2
TREE_UNSORTED = 1000  # evm_tree_from_json_dev: children keys out of order (the host parser reads it)

DIFF_NONE = -1
DIFF_RANGE_ERROR = -2

REC_BYTES = 32  # sizeof(evm_rec)

_vp = C.c_void_p
_sz = C.c_size_t
_u32 = C.c_uint32
_i = C.c_int

# name -> (restype, argtypes); every symbol include/evm.h declares.
SIGNATURES = {
    "evm_create": (_i, [_i, C.POINTER(_vp)]),
    "evm_destroy": (None, [_vp]),
    "evm_strerror": (C.c_char_p, [_i]),
    "evm_set_stream": (_i, [_vp, _vp]),
    "evm_bind_thread": (_i, [_vp]),
    "evm_get_stats": (_i, [_vp, _vp]),
    "evm_get_stream": (_vp, [_vp]),
    "evm_sync": (_i, [_vp]),
    "evm_set_option": (_i, [_vp, _i, C.c_int64]),
    "evm_test_fault": (_i, [_vp, _i]),  # include/evm_test.h (EVM_TEST_HOOKS=1 only)
    "evm_prof_enable": (_i, [_vp, _i]),
    "evm_prof_reset": (_i, [_vp]),
    "evm_cross_cell_check": (_i, [_vp, _vp, _sz, _sz, _vp, C.c_uint32, C.POINTER(C.c_int32)]),
    "evm_prof_only": (_i, [_vp, C.c_char_p]),
    "evm_prof_report": (_i, [_vp, _vp, _sz, C.POINTER(_sz)]),
    "evm_dev_alloc": (_i, [_vp, _sz, C.POINTER(_vp)]),
    "evm_dev_free": (_i, [_vp, _vp]),
    "evm_copy_h2d": (_i, [_vp, _vp, _vp, _sz]),
    "evm_copy_d2h": (_i, [_vp, _vp, _vp, _sz]),
    "evm_pack": (_i, [_vp, _vp, _sz, _sz, _vp, _vp]),
    "evm_tree_new": (_i, [_vp, _u32, C.POINTER(_vp)]),
    "evm_tree_from_leaves": (_i, [_vp, _u32, _vp, _vp, _vp, C.POINTER(_vp)]),
    "evm_tree_free": (_i, [_vp, _vp]),
    "evm_tree_from_device_leaves": (_i, [_vp, _u32, _vp, _vp, _vp, C.POINTER(_vp)]),
    "evm_tree_slice": (_i, [_vp, _vp, _u32, _u32, _vp, _vp, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "evm_tree_info": (_i, [_vp, C.POINTER(_u32), C.POINTER(C.c_uint64)]),
    "evm_tree_device": (_i, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp)]),
    "evm_tree_leaves": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "evm_tree_roots": (_i, [_vp, _vp, _vp, _vp]),
    "evm_tree_to_json": (_i, [_vp, _vp, _u32, _vp, _sz, C.POINTER(_sz)]),
    "evm_tree_to_json_batch": (_i, [_vp, _vp, _vp, _u32, _vp, _sz, _vp, C.POINTER(C.c_uint64)]),
    "evm_tree_from_json": (_i, [_vp, _u32, C.POINTER(C.c_char_p), C.POINTER(_sz), C.POINTER(_vp)]),
    "evm_merkle_insert": (_i, [_vp, _vp, _vp, _sz, _sz, _vp, C.POINTER(_vp)]),
    "evm_merkle_diff": (_i, [_vp, _vp, _vp, _vp]),
    "evm_tree_merge": (_i, [_vp, _vp, _vp, C.POINTER(_vp)]),
    "evm_receive_fold": (_i, [_vp, _vp, _sz, _sz, C.c_int64, _u32, C.c_char_p, C.c_int64, C.c_int64, _vp]),
    "evm_store_new": (_i, [_vp, _u32, C.POINTER(_vp)]),
    "evm_store_free": (_i, [_vp, _vp]),
    "evm_store_info": (_i, [_vp, C.POINTER(_u32), C.POINTER(C.c_uint64)]),
    "evm_store_tree": (_vp, [_vp]),
    "evm_store_messages": (_i, [_vp, _vp, _vp, _vp]),
    "evm_server_ingest": (_i, [_vp, _vp, _vp, _sz, _sz, _vp, C.c_uint64, _vp]),
    "evm_server_ingest_ex": (_i, [_vp, _vp, _vp, _sz, _sz, _vp, C.c_uint64, _vp, _vp]),
    "evm_pb_scan": (_i, [_i, _vp, _sz, _vp]),
    "evm_pb_split": (_i, [_i, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp]),
    "evm_pb_encode": (_i, [_i, _vp, _sz, _vp, _sz, _vp, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp, _sz, C.POINTER(_sz)]),
    "evm_pb_scan_batch": (_i, [_i, _vp, _vp, _u32, _vp, _vp]),
    "evm_pb_split_batch": (_i, [_i, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    "evm_pb_encode_requests": (_i, [_u32, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "evm_pb_encode_responses": (_i, [_u32, _vp, _vp, _u32, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _vp]),
    "evm_pb_scan_dev": (_i, [_vp, _i, _vp, _vp, _u32, _vp, _vp]),
    "evm_pb_split_dev": (_i, [_vp, _i, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "evm_pb_scan_index_dev": (_i, [_vp, _i, _vp, _vp, _u32, _vp, _vp, _vp]),
    "evm_pb_split_index_dev": (_i, [_vp, _i, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    "evm_gather_spans_dev": (_i, [_vp, _vp, _vp, _vp, _vp, _u32, _vp]),
    "evm_tree_from_json_dev": (_i, [_vp, _u32, _vp, _vp, _vp, _vp, C.POINTER(_vp)]),
    "evm_pb_encode_responses_dev": (_i, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _sz, _vp, _vp, _vp,
                                         _sz, _vp, C.POINTER(C.c_uint64)]),
    "evm_sync_create": (_i, [_vp, _vp, C.POINTER(_vp)]),
    "evm_sync_destroy": (_i, [_vp]),
    "evm_sync_round": (_i, [_vp, _vp, _vp, _u32, _i, _vp, _vp, C.POINTER(C.c_uint64)]),
    "evm_sync_fetch": (_i, [_vp, _vp]),
    "evm_sync_responses_dev": (_vp, [_vp]),
    "evm_sync_users": (_i, [_vp, _vp, _vp, _u32, _i, _vp]),
    "evm_sync_user_flag": (_i, [_vp, _u32, _i]),
    "evm_sync_user_count": (_i, [_vp, C.POINTER(_u32), C.POINTER(C.c_uint64)]),
    "evm_sync_user_keys": (_i, [_vp, _vp, _vp]),
    "evm_sync_log_add": (_i, [_vp, _vp, _sz, C.c_uint64, _vp, _vp, C.POINTER(C.c_uint64)]),
    "evm_sync_log_read": (_i, [_vp, _vp, C.c_uint64, _vp, _vp, _vp]),
    "evm_sync_next_id": (C.c_uint64, [_vp]),
    "evm_sync_timing": (_i, [_vp, _vp]),
    "evm_store_since": (_i, [_vp, _vp, _vp, _vp, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "evm_server_select": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "evm_store_select_after": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "evm_dist_unique_id": (_i, [_vp]),
    "evm_dist_init": (_i, [_vp, _vp, _i, _i, C.POINTER(_vp)]),
    "evm_dist_free": (None, [_vp, _vp]),
    "evm_dist_info": (_i, [_vp, C.POINTER(_i), C.POINTER(_i)]),
    "evm_dist_hub_new": (_i, [_i, C.POINTER(_vp)]),
    "evm_dist_hub_free": (None, [_vp]),
    "evm_dist_hub_abort": (None, [_vp]),
    "evm_dist_init_loopback": (_i, [_vp, _vp, _i, C.POINTER(_vp)]),
    "evm_dist_directory": (_i, [_vp, _vp, _vp, _sz, _sz, _u32, _vp, _vp, C.POINTER(_u32)]),
    "evm_dist_route": (_i, [_vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp, C.POINTER(C.c_uint64)]),
    "evm_dist_route_ex": (_i, [_vp, _vp, _vp, _sz, _sz, _vp, _vp, _vp, _u32, C.POINTER(C.c_uint64)]),
    "evm_dist_take": (_i, [_vp, _vp, _u32, _vp, _sz, _vp, _vp, _vp, C.c_uint64, _vp]),
    "evm_dist_ingest": (_i, [_vp, _vp, _vp, C.c_uint64, _vp]),
    "evm_dist_received": (C.c_uint64, [_vp]),
    "evm_dist_gather_roots": (_i, [_vp, _vp, _vp, _u32, _u32, _vp, _vp]),
    "evm_dist_hot_owners": (_i, [_vp, _vp, _vp, _sz, _u32, C.c_double, _vp, _u32, C.POINTER(_u32)]),
    "evm_dist_split": (_i, [_vp, _vp, _vp, _u32, _u32, C.POINTER(_u32)]),
    "evm_dist_merge_trees": (_i, [_vp, _vp, _vp, _u32, _u32, C.POINTER(_vp)]),
    "evm_dist_merge_select": (_i, [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, C.c_uint64, C.POINTER(C.c_uint64)]),
    "evm_dist_ts_dest": (_i, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "evm_dist_cell_dest": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "evm_dist_return": (_i, [_vp, _vp, _vp, _u32, _vp, _sz]),
    "evm_dist_split_winners": (_i, [_vp, _vp, _vp, _u32, _vp]),
    "evm_dist_agree_status": (_i, [_vp, _vp, C.c_int32, C.POINTER(C.c_int32)]),
    "evm_apply_batch": (
        _i,
        [_vp, _vp, _vp, _sz, _sz, _vp, _u32, _vp, _vp, _sz, _vp, _vp, _vp, C.POINTER(_vp)],
    ),
    "evm_apply_batch_async": (
        _i,
        [_vp, _vp, _vp, _sz, _sz, _vp, _u32, _vp, _vp, _sz, _vp, _vp, _sz, _sz, _vp, _vp, _vp, C.POINTER(_vp)],
    ),
    "evm_apply_wait": (_i, [_vp, _vp, C.POINTER(_vp)]),
    "evm_apply_batch_ex": (
        _i,
        [_vp, _vp, _vp, _sz, _sz, _vp, _u32, _vp, _vp, _sz, _vp, _vp, _sz, _sz, _vp, _vp, _vp, C.POINTER(_vp)],
    ),
}

_LIB = None


class EngineError(RuntimeError):
    def __init__(self, status: int, where: str):
        self.status = status
        msg = _LIB.evm_strerror(status).decode() if _LIB is not None else str(status)
        super().__init__("%s: %s (status %d)" % (where, msg, status))


def load(path: str = None):
    """Loads libevm.so (raises if absent: there is no CPU fallback).
    EVM_LIB_PATH selects another in-tree build (A/B measurements)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("EVM_LIB_PATH") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(
            "libevm.so not built (%s); run `python -c 'import __graft_entry__ as g; g.build()'`" % path
        )
    # torch bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's): load
    # it first so the process holds ONE HIP runtime, shared with libevm.
    import torch  # noqa: F401

    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(status: int, where: str):
    if status != EVM_OK:
        raise EngineError(status, where)
