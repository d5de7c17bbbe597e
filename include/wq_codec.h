/* wq_codec.h — host-side wire codec feeding the routing tick.
 *
 * Replaces, for a whole batch of received frames at once, the per-message
 *   Message::deserialize          worldql_server/src/structures/message.rs:136-142
 *     root_as_message (FlatBuffers 2.0.0 verifier)   src/flatbuffers/WorldQLFB_generated.rs:1192-1194, :986-1004
 *     MessageT -> Message decode                     message.rs:60-114
 *   sanitize_world_name           worldql_server/src/utils/world_names.rs:54-87
 * that the ZeroMQ / WebSocket ingress runs before handle_sub_messages (zeromq/incoming.rs:39-45
 * drops a frame whose deserialize fails). The decoder never allocates: it returns, per frame, the
 * fields the routing path reads (instruction, sender uuid, world-name bytes, replication, position)
 * as plain values and byte ranges into the caller's buffer.
 *
 * A Rust worldql_gpu crate binds these next to wq_router.h. Host code only: no
 * GPU is touched. Thread-safe (no shared state).
 */
#ifndef WQ_CODEC_H
#define WQ_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* wq_decoded_msg.status */
#define WQ_DEC_OK 0
#define WQ_DEC_INVALID_FLATBUFFER 1 /* DeserializeError::InvalidFlatbuffer (verifier, message.rs:137, :148) */
#define WQ_DEC_MISSING_FIELD 2      /* DecodeError::MissingRequiredField (message.rs:60-65, record.rs:33/42, entity.rs:32/36/40) */
#define WQ_DEC_BAD_UUID 3           /* Uuid::parse_str failed (uuid 0.8.2; message.rs:101, record.rs:45, entity.rs:43) */

/* Instruction codes (WorldQLFB_generated.rs:56-69); codes 13..254 decode to Unknown (instruction.rs:57-76) */
#define WQ_INSTR_AREA_SUBSCRIBE 4
#define WQ_INSTR_AREA_UNSUBSCRIBE 5
#define WQ_INSTR_GLOBAL_MESSAGE 6
#define WQ_INSTR_LOCAL_MESSAGE 7
#define WQ_INSTR_UNKNOWN 255

typedef struct wq_decoded_msg {
    int32_t status;         /* WQ_DEC_*; the other fields are meaningful only when WQ_DEC_OK */
    uint8_t instruction;    /* 0..12, or 255 (Unknown) */
    uint8_t replication;    /* 0 ExceptSelf, 1 IncludingSelf, 2 OnlySelf (unknown codes -> 0, replication.rs:34-43) */
    uint8_t has_position;   /* Message.position is Some */
    uint8_t has_parameter;  /* Message.parameter is Some */
    uint8_t sender_uuid[16];/* Uuid bytes, big-endian as written (RFC 4122 text order) */
    double position[3];     /* x, y, z (Vec3d, little-endian f64) */
    uint32_t world_off;     /* world_name: byte range [world_off, world_off + world_len) of this frame */
    uint32_t world_len;
    uint32_t param_off;     /* parameter: byte range of this frame (has_parameter) */
    uint32_t param_len;
    uint32_t n_records;     /* records / entities decoded and validated (not returned) */
    uint32_t n_entities;
} wq_decoded_msg;

/* Decode n frames: frame i is data[offsets[i] .. offsets[i + 1]) (offsets has n + 1 entries).
 * n_threads <= 0: a default based on n and the host's cores. Returns 0, or a negative code for
 * invalid arguments (-1). A frame that fails to decode is reported in its status, never fatal. */
int wq_decode_messages(const uint8_t* data, const uint64_t* offsets, size_t n, wq_decoded_msg* out,
                       int n_threads);

/* sanitize_world_name (world_names.rs:54-87) of the UTF-8 bytes name[0 .. len). Returns 0 and the
 * sanitized name in out[0 .. *out_len) (not NUL-terminated; at most 63 bytes, so cap >= 63 always
 * suffices), or the SanitizeError variant (world_names.rs:89-105): */
#define WQ_SAN_IS_GLOBAL_WORLD 1
#define WQ_SAN_ZERO_LENGTH 2
#define WQ_SAN_INVALID_START 3
#define WQ_SAN_INVALID_CHARS 4
#define WQ_SAN_TOO_LONG 5
int wq_sanitize_world_name(const char* name, size_t len, char* out, size_t cap, size_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* WQ_CODEC_H */
