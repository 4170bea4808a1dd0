/*
 * plato_ingest.h — native ingestion of Plato client payloads (host side).
 *
 * A client payload reaches the server as the bytes of pickle.dumps(state_dict)
 * (socket.io chunks joined at plato/servers/base.py:821, or the
 * comm_simulation file read at :791-792) and is turned back into tensors by
 * pickle.loads (:822).  For a ResNet-18 payload that costs ~32 ms of Python
 * per client.  This library parses the same bytes in C++,
 * without executing anything: it recognises only the opcodes and callables a
 * pickled state_dict of CPU tensors uses
 *
 *   collections.OrderedDict()                      (or a plain dict)
 *   torch._utils._rebuild_tensor_v2(storage, offset, size, stride, grad, hooks[, meta])
 *   torch.storage._load_from_bytes(<legacy torch.save record>)
 *
 * and refuses anything else (PLATO_INGEST_EUNSUPPORTED).  The legacy record
 * is (pickles of) magic number, protocol 1001, sys info, a persistent-id tuple
 * ('storage', torch.<T>Storage, key, location, numel, view), the key list,
 * then per storage an int64 element count and the raw little-endian data.
 *
 * Reference interface replaced: pickle.loads of a payload at
 * plato/servers/base.py:822 (and pickle.load at :791-792), followed by the
 * engine's per-tensor pack into the flat arena.
 */
#ifndef PLATO_INGEST_H
#define PLATO_INGEST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLATO_INGEST_MAX_DIMS 8

#define PLATO_INGEST_EINVAL (-1)       /* bad argument                          */
#define PLATO_INGEST_EFORMAT (-3)      /* malformed or truncated pickle         */
#define PLATO_INGEST_EUNSUPPORTED (-4) /* valid pickle outside the accepted set */
#define PLATO_INGEST_ECAPACITY (-5)    /* more tensors than the output array,
                                          or a destination buffer too small     */
#define PLATO_INGEST_ENOCODEC (-6)     /* libzstd.so.1 not available            */
#define PLATO_INGEST_EUNKNOWNSIZE (-7) /* zstd frame without a content size     */
#define PLATO_INGEST_EIO (-8)          /* read error or short file              */

/* dtype codes (torch storage classes) */
#define PLATO_DT_F32 0  /* FloatStorage    */
#define PLATO_DT_I64 1  /* LongStorage     */
#define PLATO_DT_F64 2  /* DoubleStorage   */
#define PLATO_DT_F16 3  /* HalfStorage     */
#define PLATO_DT_BF16 4 /* BFloat16Storage */
#define PLATO_DT_I32 5  /* IntStorage      */
#define PLATO_DT_I16 6  /* ShortStorage    */
#define PLATO_DT_I8 7   /* CharStorage     */
#define PLATO_DT_U8 8   /* ByteStorage     */
#define PLATO_DT_BOOL 9 /* BoolStorage     */

typedef struct {
  uint64_t name_offset;   /* key bytes (UTF-8) inside the input buffer */
  uint32_t name_len;
  int32_t dtype;          /* PLATO_DT_*                                 */
  int32_t ndim;
  int32_t contiguous;     /* 1 if stride is C-contiguous for shape      */
  int64_t shape[PLATO_INGEST_MAX_DIMS];
  int64_t stride[PLATO_INGEST_MAX_DIMS];
  uint64_t numel;
  uint64_t storage_offset; /* elements                                  */
  uint64_t storage_numel;
  uint64_t data_offset;    /* byte offset of storage element 0 in the buffer */
  int32_t storage_id;      /* tensors sharing a storage share this id    */
  int32_t element_size;
} plato_ingest_tensor;

/* Thread-local message for the last failure ("" if none). */
const char* plato_ingest_last_error(void);

/*
 * Parse pickle.dumps(state_dict) bytes.  Writes up to max_tensors entries in
 * the dict's insertion order and returns the number of tensors (>= 0), or a
 * negative PLATO_INGEST_E* code.  Reads only [buf, buf + len).
 */
int plato_ingest_parse(const uint8_t* buf, size_t len, plato_ingest_tensor* out, int max_tensors);

/*
 * Gather parsed tensors into a flat destination: tensor i (logical C order,
 * strided sources allowed) is written as its dtype's bytes at
 * dst + dst_byte_offset[i].  Contiguous tensors are memcpy'd; the copy is
 * spread over `threads` host threads (<= 0: hardware concurrency).
 */
int plato_ingest_gather(const uint8_t* buf, size_t len, const plato_ingest_tensor* t, int n,
                        const uint64_t* dst_byte_offset, uint8_t* dst, size_t dst_len, int threads);

/* Packs n contiguous host pieces into one destination (the engine's pinned
 * staging arena) on the same thread pool: piece i is bytes[i] bytes copied
 * from src[i] to dst + dst_off[i].  It replaces the per-tensor pack of a CPU
 * state_dict into the flat arena before its H2D copy (the reference keeps the
 * tensors apart and reads them one by one in aggregate_deltas,
 * plato/servers/fedavg.py:148-154).  threads <= 0: up to 16 pool threads.
 * Returns 0, PLATO_INGEST_EINVAL or PLATO_INGEST_ECAPACITY (a piece outside
 * dst). */
int plato_ingest_pack(const void* const* src, const uint64_t* bytes, const uint64_t* dst_off, int n, void* dst,
                      size_t dst_len, int threads);

/*
 * Join a payload's transport chunks (socket.io delivers 1 MiB chunks that the
 * server concatenates with b"".join before unpickling, plato/servers/base.py:
 * 813-822) into dst, on the same thread pool as plato_ingest_gather: one
 * parallel copy instead of Python's single-threaded join.  dst may be the
 * buffer plato_ingest_parse then reads.
 */
int plato_ingest_join(const uint8_t* const* chunks, const size_t* lens, int n, uint8_t* dst, size_t dst_len,
                      int threads);

/*
 * Read the first len bytes of an open file (offset 0, pread, file position
 * untouched) into dst, in 4 MiB pieces on the same thread pool.  Under
 * comm_simulation (Plato's default, plato/clients/base.py:92-96) a client's
 * payload reaches the server as a file it pickle.dump'ed
 * (clients/base.py:372-386) and the server pickle.load's it
 * (plato/servers/base.py:791-792); this is the read half of that, parse and
 * gather being the rest.  Returns len, or PLATO_INGEST_EIO.
 */
int64_t plato_ingest_read_fd(int fd, uint8_t* dst, size_t len, int threads);

/*
 * zstd-compressed payloads.  Plato's model_compress outbound processor sends
 * zstd.compress(pickle.dumps(state_dict), level)
 * (plato/processors/model_compress.py:25) and the server's model_decompress
 * inbound processor runs pickle.loads(zstd.decompress(data))
 * (plato/processors/model_decompress.py:24).  These entry points replace the
 * zstd.decompress half (the pickle half is plato_ingest_parse / _gather) with
 * the system libzstd.so.1, bound at first use (dlopen); without it they
 * return PLATO_INGEST_ENOCODEC.  Standard zstd frames (RFC 8878), one or
 * several concatenated.
 */
/* 1 if libzstd.so.1 could be bound, else 0 (plato_ingest_last_error says why). */
int plato_ingest_zstd_available(void);

/* Total decompressed size of the frames in [src, src + len), or
 * PLATO_INGEST_EUNKNOWNSIZE when a frame header omits it, or an error. */
int64_t plato_ingest_zstd_content_size(const uint8_t* src, size_t len);

/* Decompress into dst (cap bytes); returns the decompressed size or an error
 * (PLATO_INGEST_ECAPACITY if cap is too small). */
int64_t plato_ingest_zstd_decompress(const uint8_t* src, size_t len, uint8_t* dst, size_t cap);

/* Worst-case compressed size of len bytes (0 without libzstd). */
size_t plato_ingest_zstd_bound(size_t len);

/* One zstd frame (with content size) of [src, src + len) at `level`: what the
 * clients' model_compress sends.  Returns the frame size or an error. */
int64_t plato_ingest_zstd_compress(const uint8_t* src, size_t len, uint8_t* dst, size_t cap, int level);

#ifdef __cplusplus
}
#endif

#endif /* PLATO_INGEST_H */
