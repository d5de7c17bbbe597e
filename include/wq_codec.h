/* wq_codec.h — host-side wire codec either side of the routing tick.
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

/* ---- serialize: the egress half of F4 -------------------------------------------------------
 * Replaces Message::serialize (structures/message.rs:120-134): Message -> MessageT (message.rs:28-52,
 * record.rs:18-26, entity.rs:17-25), MessageT::pack (WorldQLFB_generated.rs:1133-1173, RecordT /
 * EntityT::pack :619-645 / :838-864) into a reset FlatBufferBuilder (flatbuffers 2.0.0, Cargo.lock:
 * 347-349), finish(root, None). The bytes are the ones that builder lays down: back-to-front, fields
 * added in the generated create() order (:1045-1055, :449-457, :668-676), scalars equal to their
 * default (Heartbeat, ExceptSelf) omitted, vtables shared within the frame. PeerMap::broadcast_to
 * serializes a routed message once for all its recipients (transport/peer_map.rs:22-40); the batch
 * entry point does that for a whole tick's messages on the host's cores. Host code only. */

/* A Record (structures/record.rs:8-15) or an Entity (entity.rs:7-14). Strings are UTF-8 bytes
 * (not NUL-terminated). For an Entity the position is not optional and has_position is ignored. */
typedef struct wq_record_in {
    uint8_t uuid[16];          /* written as uuid 0.8.2's to_string(): lower-case hyphenated */
    uint8_t has_position;
    uint8_t has_data;          /* data: Option<String> */
    uint8_t has_flex;          /* flex: Option<Bytes> */
    uint8_t pad_[5];
    double position[3];
    const char* world_name;
    uint64_t world_len;
    const char* data;
    uint64_t data_len;
    const uint8_t* flex;
    uint64_t flex_len;
} wq_record_in;

/* A Message (structures/message.rs:13-24). */
typedef struct wq_message_in {
    uint8_t instruction;       /* wire code: 0..12, or 255 (Unknown, the Default) */
    uint8_t replication;       /* 0 ExceptSelf, 1 IncludingSelf, 2 OnlySelf */
    uint8_t has_position;
    uint8_t has_parameter;
    uint8_t has_flex;
    uint8_t pad_[3];
    uint8_t sender_uuid[16];
    double position[3];
    const char* parameter;
    uint64_t parameter_len;
    const char* world_name;
    uint64_t world_len;
    const uint8_t* flex;
    uint64_t flex_len;
    const wq_record_in* records;
    uint64_t n_records;
    const wq_record_in* entities;
    uint64_t n_entities;
} wq_message_in;

#define WQ_SER_INVALID_ARG -1
#define WQ_SER_SHORT -2        /* out has fewer than the needed bytes: the size is reported, nothing else */
#define WQ_SER_INVALID_UTF8 -3 /* a string field is not UTF-8 (a Rust String cannot hold it) */
#define WQ_SER_TOO_LARGE -4    /* the builder's 2 GiB limit (it panics there; 1 GiB frames at most) */

/* One frame into out[0 .. *out_len). On WQ_SER_SHORT, *out_len is the size needed. */
int wq_serialize_message(const wq_message_in* m, uint8_t* out, size_t cap, size_t* out_len);

/* n frames back to back: frame i is out[offsets[i] .. offsets[i + 1]) (offsets has n + 1 entries,
 * always filled when the messages are valid). WQ_SER_SHORT when offsets[n] > cap; on any other
 * error the first failing message's code is returned. n_threads <= 0: a default from n and the
 * host's cores. */
int wq_serialize_messages(const wq_message_in* msgs, size_t n, uint8_t* out, size_t cap, uint64_t* offsets,
                          int n_threads);

/* An upper bound of the bytes wq_serialize_messages writes for these messages. With out holding
 * at least this many bytes the frames are packed in place (one pass, no staging copy). */
size_t wq_serialize_bound(const wq_message_in* msgs, size_t n);

#ifdef __cplusplus
}
#endif
#endif /* WQ_CODEC_H */
