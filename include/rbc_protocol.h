/* rbc_protocol.h -- the RBC state machine above the data path (SURVEY §8f
 * rank 1-3), in C++ behind a C ABI because the reference's own language (Go)
 * is absent from this image.
 *
 * Mirrors rbc/rbc.go:9-100 (NewRBC, HandleMessage, handleValueRequest /
 * handleEchoRequest / handleReadyRequest, Value, Messages) and the request
 * types of rbc/request.go:9-21, exchanged as pb.Message (pb/message.proto:11-35;
 * the generated code carries RBC.type as field 2, pb/message.pb.go:182-183).
 *
 * Protocol (docs/RBC-EN.md, HBBFT): the proposer sends VAL(h, b_j, s_j) to
 * node j; a node multicasts ECHO(h, b_i, s_i) for the VAL it received; an ECHO
 * from node j counts iff validateMessage proves s_j at leaf j under h; with
 * N-f valid ECHOs for h the node interpolates and, when the re-encoded root
 * matches h, multicasts READY(h); f+1 READY(h) make it multicast READY(h) too;
 * 2f+1 READY(h) plus N-2f valid ECHOs deliver the value.
 *
 * Payload codec (unpinned by the reference: its handlers are stubs): the
 * request structs marshaled by Go encoding/json -- fields in struct order,
 * []byte as standard base64, nil slices as null, EchoRequest's embedded
 * ValRequest promoted: {"RootHash":"..","Branch":"..","Block":[".."]} and
 * {"RootHash":".."}.  Branch is the Go flat form (the non-empty siblings,
 * leaf to root) that rbc_validate_message takes.
 *
 * GPU work (shard + commit, validateMessage, interpolate) is submitted to an
 * rbc_batcher without blocking, so every instance and node of the process
 * shares launches; rbc_node_progress completes it.  Node indices are the
 * positions in the sorted member list (= Merkle leaf index). */
#ifndef RBC_PROTOCOL_H
#define RBC_PROTOCOL_H

#include <stddef.h>
#include <stdint.h>

#include "rbc_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RBC_MSG_VAL 0   /* pb.RBC_VAL   */
#define RBC_MSG_ECHO 1  /* pb.RBC_ECHO  */
#define RBC_MSG_READY 2 /* pb.RBC_READY */
#define RBC_ERR_PROTOCOL (-20) /* malformed or out-of-protocol message */

/* ---- codec (host only, no GPU) ------------------------------------------- */
/* pb.Message{rbc: pb.RBC{payload, type}} (signature/timestamp unset).
 * Returns the encoded size; writes only when it fits in cap. */
size_t rbc_pb_encode_rbc(int type, const uint8_t *payload, size_t payload_len, uint8_t *out, size_t cap);
/* Parse a pb.Message carrying an RBC: *type, *payload (points into msg). */
int rbc_pb_decode_rbc(const uint8_t *msg, size_t len, int *type, const uint8_t **payload, size_t *payload_len);
/* Go encoding/json of ValRequest / EchoRequest (one shape, block = Block[0];
 * block_len 0 -> "Block":null) and ReadyRequest.  Returns the size; writes
 * only when it fits. */
size_t rbc_json_encode_val(const uint8_t *root, size_t root_len, const uint8_t *branch, size_t branch_len,
                           const uint8_t *block, size_t block_len, uint8_t *out, size_t cap);
size_t rbc_json_encode_ready(const uint8_t *root, size_t root_len, uint8_t *out, size_t cap);
/* json.Unmarshal of the same shapes (keys case-insensitive, unknown keys
 * skipped): RootHash must be 32 bytes and Block hold exactly one shard.
 * RBC_ERR_PROTOCOL when malformed; RBC_ERR_INVALID_ARG (lens set) when a
 * buffer is short. */
int rbc_json_decode_val(const uint8_t *json, size_t len, uint8_t *root_out, uint8_t *branch_out, size_t branch_cap,
                        size_t *branch_len, uint8_t *block_out, size_t block_cap, size_t *block_len);
int rbc_json_decode_ready(const uint8_t *json, size_t len, uint8_t *root_out);

/* ---- device-side marshaling (the proposer's per-recipient VAL send path) --
 * For every instance i and row j, writes the pb.Message bytes of VAL / ECHO
 * (type) carrying (roots[i], flat branch j, shard j) -- byte-identical to
 * rbc_pb_encode_rbc(type, rbc_json_encode_val(...)) -- to
 * out + (i*n + j)*out_pitch, and out_lens[i*n + j] = its size (nullable).
 * Inputs in the rbc_dev_* layout (rbc_gpu.h): shards [count][n][shard_pitch],
 * branches [count][n][d][32], roots [count][32].  out_pitch % 16 == 0 and
 * >= round_up(rbc_val_message_size(n, S_max, 0, type), 16); bytes past a
 * message up to the next 16 are zeroed. */
int rbc_dev_marshal_val(rbc_ctx *ctx, void *stream, int count, int type, const uint8_t *shards,
                        uint32_t shard_pitch, const uint32_t *shard_lens, uint32_t uniform_shard_len,
                        const uint8_t *branches, const uint8_t *roots, uint8_t *out, uint64_t out_pitch,
                        uint32_t *out_lens);
/* Size of that message for shard length S at leaf `index` of an n-node tree. */
size_t rbc_val_message_size(int n, uint32_t shard_len, uint32_t index, int type);

/* The proposer's send path in one call (the gap at
 * conn.go:182-208, where Broadcaster.Broadcast sends one message to all while
 * VAL differs per recipient): shard + commit `count` proposals (host values),
 * marshal every per-recipient VAL on the device, and move the finished
 * pb.Message bytes to the caller's ring in ONE device-to-host copy:
 * msgs [count][n][msg_pitch] (message (i, j) for member j at
 * msgs + (i*n + j)*msg_pitch, msg_lens [count][n] bytes), roots_out
 * [count][32] (nullable).  msg_pitch % 16 == 0 and >= the largest
 * rbc_val_message_size(n, S_max, index, RBC_MSG_VAL).  Ring memory from
 * rbc_host_alloc is written directly by the DMA engine (no staging copy);
 * a gRPC writer sends msgs[i][j][:len] to member j with a pass-through codec
 * (INTEGRATION.md).  Asynchronous: complete with rbc_wait / rbc_poll. */
int rbc_shard_commit_val(rbc_ctx *ctx, int count, const uint8_t *const *values, const size_t *value_lens,
                         uint8_t *msgs, size_t msg_pitch, uint32_t *msg_lens, uint8_t *roots_out,
                         uint64_t *ticket);

/* ---- RBC instance (one proposer's broadcast, seen at one node) ----------- */
typedef struct rbc_node rbc_node;
/* NewRBC (rbc/rbc.go:38). */
int rbc_node_create(rbc_batcher *batcher, int n, int f, int self, int proposer, rbc_node **out);
void rbc_node_destroy(rbc_node *node); /* waits for its outstanding GPU work */
/* Proposer only: shard + commit `value` (copied), then VAL(h, b_j, s_j) to every j.
 * The broadcast payload is framed as [u64 little-endian len][value] (len 0 is
 * allowed), so rbc_node_value returns exactly these bytes. */
int rbc_node_propose(rbc_node *node, const uint8_t *value, size_t len);
/* HandleMessage (rbc/rbc.go:47): a marshaled pb.Message from node `sender`.
 * Parses and submits its GPU check; the outcome applies in rbc_node_progress.
 * Returns RBC_ERR_PROTOCOL for a malformed, duplicate or out-of-protocol
 * message (it is dropped and counted). */
int rbc_node_handle_message(rbc_node *node, int sender, const uint8_t *msg, size_t len);
/* Completes submitted GPU work in order and advances the state machine:
 * wait = 0 applies only what is done, wait = 1 blocks until all is done.
 * *pending_out (nullable) = submissions still outstanding. */
int rbc_node_progress(rbc_node *node, int wait, int *pending_out);
/* Messages (rbc/rbc.go:74): pops the next outgoing message into buf;
 * *to = recipient index, or -1 for every node but this one (a node applies
 * its own ECHO/READY locally).  *len = 0: queue empty.  cap too small:
 * returns RBC_ERR_INVALID_ARG with *len = the size needed (message kept). */
int rbc_node_next_message(rbc_node *node, int *to, uint8_t *buf, size_t cap, size_t *len);
/* Value (rbc/rbc.go:69): *delivered = 1 once decided; the value is the
 * proposer's bytes, unframed from the interpolated k*S bytes.  A delivered
 * payload whose frame length exceeds it (a Byzantine proposer: every honest
 * node sees the same bytes) returns RBC_ERR_PROTOCOL with *delivered = 1 and
 * *len = 0.  buf NULL with cap 0: only *len and *delivered are set.
 * rbc_node_create requires n >= 3f + 1 (HBBFT quorum intersection). */
int rbc_node_value(rbc_node *node, uint8_t *buf, size_t cap, size_t *len, int *delivered);
/* Valid ECHOs and READYs for the leading root, READY sent (0/1), messages
 * rejected (bad proof, wrong sender, malformed, duplicate). */
int rbc_node_stats(rbc_node *node, int *echoes, int *readies, int *ready_sent, int *rejected);

#ifdef __cplusplus
}
#endif
#endif
