"""ctypes binding of ``librbc_gpu.so`` (include/rbc_gpu.h).

The product path is the HIP library; there is no CPU fallback.  Importing
this module without the built library raises immediately.
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# RBC_GPU_LIB: another build of the same ABI (an A/B candidate from tools/build_ab.sh, or a
# test-only mutant from tests/mutants that the guard tests expect to FAIL); the bench line
# records the file actually mapped (rbc_library_path, dladdr) so a run says what it measured.
# RBC_GPU_LIB_AB is round 3's name for the same override (archived run scripts still set it).
LIB_PATH = (os.environ.get("RBC_GPU_LIB") or os.environ.get("RBC_GPU_LIB_AB")
            or os.path.join(_HERE, "librbc_gpu.so"))
INCLUDE_DIR = os.path.join(os.path.dirname(_HERE), "include")
HEADER_PATH = os.path.join(INCLUDE_DIR, "rbc_gpu.h")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
        "(the RBC data path has no CPU fallback)")

lib = ctypes.CDLL(LIB_PATH)

u8p = POINTER(c_uint8)
u32p = POINTER(c_uint32)
i32p = POINTER(c_int32)
szp = POINTER(c_size_t)
u8pp = POINTER(u8p)


class RxBatch(ctypes.Structure):
    """rbc_rx_batch (include/rbc_gpu.h): one batch of rbc_dev_receive_step."""
    _fields_ = [("count", c_int), ("shards", c_void_p), ("shard_pitch", c_uint32), ("shard_lens", c_void_p),
                ("uniform_shard_len", c_uint32), ("branches", c_void_p), ("roots", c_void_p),
                ("present", c_void_p), ("valid", c_void_p), ("leaves", c_void_p), ("values_out", c_void_p),
                ("value_pitch", c_uint32), ("digests", c_void_p), ("status", c_void_p), ("verified", c_int)]


class RxMarks(ctypes.Structure):
    """rbc_rx_marks (include/rbc_gpu.h): timing events of rbc_dev_receive_step."""
    _fields_ = [("hashed", c_void_p), ("decode_begin", c_void_p), ("decoded", c_void_p), ("hash_begin", c_void_p),
                ("rows_hashed", c_void_p), ("prev_released", c_void_p)]


_SIGS = {
    "rbc_strerror": (c_char_p, [c_int]),
    "rbc_abi_version": (c_int, []),
    "rbc_ctx_verify_form": (c_int, [c_void_p, c_uint32, POINTER(c_int)]),
    "rbc_library_path": (c_int, [c_char_p, c_size_t]),
    "rbc_device_count": (c_int, [POINTER(c_int)]),
    "rbc_ctx_create": (c_int, [c_int, c_int, c_int, POINTER(c_void_p)]),
    "rbc_ctx_destroy": (None, [c_void_p]),
    "rbc_ctx_params": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "rbc_ctx_encode_matrix": (c_int, [c_void_p, c_void_p]),
    "rbc_ctx_set_codec": (c_int, [c_void_p, c_int]),
    "rbc_ctx_set_wave_priority": (c_int, [c_void_p, c_int, c_int]),
    "rbc_ctx_set_decode_priority": (c_int, [c_void_p, c_int, c_int]),
    "rbc_ctx_set_recheck": (c_int, [c_void_p, c_int]),
    "rbc_ctx_codec": (c_int, [c_void_p, POINTER(c_int)]),
    "rbc_dev_malloc": (c_int, [c_int, c_size_t, POINTER(c_void_p)]),
    "rbc_dev_free": (c_int, [c_void_p]),
    "rbc_dev_memset": (c_int, [c_void_p, c_int, c_size_t]),
    "rbc_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_size_t]),
    "rbc_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_size_t]),
    "rbc_host_alloc": (c_int, [c_size_t, POINTER(c_void_p)]),
    "rbc_host_free": (c_int, [c_void_p]),
    "rbc_stream_create": (c_int, [c_int, POINTER(c_void_p)]),
    "rbc_stream_create_priority": (c_int, [c_int, c_int, POINTER(c_void_p)]),
    "rbc_stream_destroy": (c_int, [c_void_p]),
    "rbc_stream_sync": (c_int, [c_void_p]),
    "rbc_event_create": (c_int, [POINTER(c_void_p)]),
    "rbc_event_destroy": (c_int, [c_void_p]),
    "rbc_event_record": (c_int, [c_void_p, c_void_p]),
    "rbc_event_elapsed_ms": (c_int, [c_void_p, c_void_p, POINTER(c_float)]),
    "rbc_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "rbc_device_sync": (c_int, [c_int]),
    "rbc_device_mem_info": (c_int, [c_int, szp, szp]),
    "rbc_dev_encode": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint64, c_void_p, c_uint32, c_void_p,
                               c_uint32]),
    "rbc_dev_leaves": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p]),
    "rbc_dev_merkle_build": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "rbc_dev_shard_commit": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint64, c_void_p, c_uint32, c_void_p,
                                     c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rbc_dev_verify": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "rbc_dev_interpolate": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint32, c_void_p, c_uint32, c_void_p,
                                    c_void_p, c_int, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
    "rbc_dev_receive_step": (c_int, [c_void_p, c_void_p, POINTER(RxBatch), POINTER(RxBatch), POINTER(RxMarks)]),
    "rbc_dev_inject_faults": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_uint32, c_void_p]),
    "rbc_shard_commit": (c_int, [c_void_p, c_int, c_void_p, szp, c_void_p, c_size_t, u32p, c_void_p, c_void_p,
                                 POINTER(c_uint64)]),
    "rbc_validate_batch": (c_int, [c_void_p, c_int, c_void_p, szp, u32p, c_void_p, szp, c_void_p, c_void_p,
                                   POINTER(c_uint64)]),
    "rbc_interpolate_batch": (c_int, [c_void_p, c_int, c_void_p, c_size_t, szp, c_void_p, c_void_p, c_void_p,
                                      c_size_t, c_void_p, i32p, POINTER(c_uint64)]),
    "rbc_wait": (c_int, [c_void_p, c_uint64]),
    "rbc_poll": (c_int, [c_void_p, c_uint64, POINTER(c_int)]),
    "rbc_shard": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, szp, c_void_p, c_void_p]),
    "rbc_validate_message": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_uint32,
                                     POINTER(c_int)]),
    "rbc_interpolate": (c_int, [c_void_p, c_void_p, c_void_p, szp, c_void_p, c_size_t, szp, c_void_p]),
    "rbc_batcher_create": (c_int, [c_void_p, c_int, c_int, POINTER(c_void_p)]),
    "rbc_batcher_destroy": (None, [c_void_p]),
    "rbc_batcher_shard": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, szp, c_void_p, c_void_p,
                                  POINTER(c_uint64)]),
    "rbc_batcher_validate": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_uint32,
                                     POINTER(c_int), POINTER(c_uint64)]),
    "rbc_batcher_interpolate": (c_int, [c_void_p, c_void_p, c_void_p, szp, c_void_p, c_size_t, szp, c_void_p,
                                        POINTER(c_uint64)]),
    "rbc_batcher_wait": (c_int, [c_void_p, c_uint64]),
    "rbc_batcher_poll": (c_int, [c_void_p, c_uint64, POINTER(c_int)]),
    "rbc_batcher_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
    "rbc_batcher_set_validate": (c_int, [c_void_p, c_int, c_size_t]),
    "rbc_batcher_set_keep": (c_int, [c_void_p, c_size_t]),
    "rbc_batcher_keep_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64),
                                       POINTER(c_uint64)]),
    "rbc_ctx_device": (c_int, [c_void_p, POINTER(c_int)]),
    "rbc_validate_packed": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, POINTER(c_uint64)]),
    "rbc_validate_packed_leaves": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, POINTER(c_uint64)]),
    "rbc_validate_packed_keep": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                         POINTER(c_uint64)]),
    "rbc_interpolate_batch_kept": (c_int, [c_void_p, c_int, c_void_p, szp, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p, i32p, POINTER(c_uint64)]),
    "rbc_interpolate_batch_verified": (c_int, [c_void_p, c_int, c_void_p, c_size_t, szp, c_void_p, c_void_p,
                                               c_void_p, c_void_p, c_size_t, c_void_p, i32p, POINTER(c_uint64)]),
    "rbc_receive_batch": (c_int, [c_void_p, c_int, c_void_p, c_size_t, szp, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_size_t, c_void_p, i32p, POINTER(c_uint64)]),
    "rbc_batcher_validate_leaf": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_uint32,
                                          POINTER(c_int), c_void_p, POINTER(c_uint64)]),
    "rbc_batcher_interpolate_verified": (c_int, [c_void_p, c_void_p, c_void_p, szp, c_void_p, c_void_p, c_size_t,
                                                 szp, c_void_p, POINTER(c_uint64)]),
    "rbc_rs_new": (c_int, [c_int, c_int, c_int, POINTER(c_void_p)]),
    "rbc_rs_free": (None, [c_void_p]),
    "rbc_rs_encode": (c_int, [c_void_p, c_void_p, szp, c_int]),
    "rbc_rs_verify": (c_int, [c_void_p, c_void_p, szp, c_int, POINTER(c_int)]),
    "rbc_rs_reconstruct": (c_int, [c_void_p, c_void_p, szp, c_int]),
    "rbc_rs_reconstruct_data": (c_int, [c_void_p, c_void_p, szp, c_int]),
    "rbc_rs_split": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, szp]),
    "rbc_rs_join": (c_int, [c_void_p, c_void_p, szp, c_int, c_size_t, c_void_p]),
    "rbc_rs_update": (c_int, [c_void_p, c_void_p, szp, c_int, c_void_p, szp, c_int]),
    "rbc_comm_unique_id": (c_int, [c_void_p]),
    "rbc_comm_init": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "rbc_comm_destroy": (c_int, [c_void_p]),
    "rbc_dev_allgather_roots": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "rbc_dev_allgather_records": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                          c_void_p]),
    "rbc_comm_info": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int), c_char_p, c_size_t,
                              POINTER(c_int), c_char_p, c_size_t]),
    "rbc_device_pci_bus_id": (c_int, [c_int, c_char_p, c_int]),
    "rbc_acs_partition": (c_int, [c_int, c_int, c_int, POINTER(c_int), POINTER(c_int)]),
    "rbc_acs_max_share": (c_int, [c_int, c_int, POINTER(c_int)]),
    "rbc_acs_assemble": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, POINTER(c_int)]),
    "rbc_dev_fill_random": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_uint64]),
    "rbc_dev_count_mismatch": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_uint64,
                                       c_void_p]),
    "rbc_dev_count_mismatch_rows": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint32, c_int, c_uint32, c_void_p,
                                            c_uint64, c_uint32, c_uint64, c_void_p]),
    "rbc_dev_poison_rows": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint32, c_int, c_void_p, c_void_p,
                                    c_uint64, c_uint64]),
    # include/rbc_protocol.h
    "rbc_pb_encode_rbc": (c_size_t, [c_int, c_void_p, c_size_t, c_void_p, c_size_t]),
    "rbc_pb_decode_rbc": (c_int, [c_void_p, c_size_t, POINTER(c_int), POINTER(c_void_p), szp]),
    "rbc_json_encode_val": (c_size_t, [c_void_p, c_size_t, c_void_p, c_size_t, c_void_p, c_size_t, c_void_p,
                                       c_size_t]),
    "rbc_json_encode_ready": (c_size_t, [c_void_p, c_size_t, c_void_p, c_size_t]),
    "rbc_json_decode_val": (c_int, [c_void_p, c_size_t, c_void_p, c_void_p, c_size_t, szp, c_void_p, c_size_t,
                                    szp]),
    "rbc_json_decode_ready": (c_int, [c_void_p, c_size_t, c_void_p]),
    "rbc_dev_marshal_val": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_uint32, c_void_p, c_uint32,
                                    c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rbc_val_message_size": (c_size_t, [c_int, c_uint32, c_uint32, c_int]),
    "rbc_shard_commit_val": (c_int, [c_void_p, c_int, c_void_p, szp, c_void_p, c_size_t, u32p, c_void_p,
                                     POINTER(c_uint64)]),
    "rbc_node_create": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "rbc_node_destroy": (None, [c_void_p]),
    "rbc_node_propose": (c_int, [c_void_p, c_void_p, c_size_t]),
    "rbc_node_handle_message": (c_int, [c_void_p, c_int, c_void_p, c_size_t]),
    "rbc_node_progress": (c_int, [c_void_p, c_int, POINTER(c_int)]),
    "rbc_node_next_message": (c_int, [c_void_p, POINTER(c_int), c_void_p, c_size_t, szp]),
    "rbc_node_value": (c_int, [c_void_p, c_void_p, c_size_t, szp, POINTER(c_int)]),
    "rbc_node_stats": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
}

for _name, (_res, _args) in _SIGS.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


def header_functions(path: str = None):
    """Every function the C-ABI headers declare (all of include/*.h, or one
    header), for the export test."""
    paths = [path] if path else sorted(os.path.join(INCLUDE_DIR, f) for f in os.listdir(INCLUDE_DIR)
                                       if f.endswith(".h"))
    names = set()
    for p in paths:
        text = open(p).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names.update(re.findall(r"\b(rbc_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


# status codes (include/rbc_gpu.h)
RBC_OK = 0
RBC_ERR_INV_SHARD_NUM = -1
RBC_ERR_MAX_SHARD_NUM = -2
RBC_ERR_TOO_FEW_SHARDS = -3
RBC_ERR_SHARD_NO_DATA = -4
RBC_ERR_SHARD_SIZE = -5
RBC_ERR_SHORT_DATA = -6
RBC_ERR_RECONSTRUCT_REQUIRED = -7
RBC_ERR_ROOT_MISMATCH = -8
RBC_ERR_DEVICE = -9
RBC_ERR_INVALID_ARG = -10
RBC_ERR_SINGULAR = -11
RBC_ERR_NO_COMM = -12
RBC_ERR_INVALID_INPUT = -13
RBC_ERR_PROTOCOL = -20  # include/rbc_protocol.h

# pb.RBC type (pb/message.proto:30-34)
RBC_MSG_VAL, RBC_MSG_ECHO, RBC_MSG_READY = 0, 1, 2


class RBCError(Exception):
    def __init__(self, code: int, where: str = ""):
        self.code = code
        msg = lib.rbc_strerror(code).decode()
        super().__init__(f"{where}: {msg} ({code})" if where else f"{msg} ({code})")


def check(code: int, where: str = "") -> None:
    if code != RBC_OK:
        raise RBCError(code, where)
