/* dlio — native TFRecord batch reader (host C++, no GPU, no torch types).
 *
 * Replaces the input pipeline of the reference, utils/data_loader.py:7-40:
 *   TFRecordDataset(files) -> map(_parse_function, num_parallel_calls=10)
 *     -> shuffle(batch_size * 10) -> batch(batch_size, drop_remainder=True)
 *     -> repeat(epochs)                                  (:29-40)
 * with _parse_function's FixedLenFeature spec (:7-26): every record must carry each
 * configured feature with exactly `size` values of the configured type, else the read
 * fails (TF raises InvalidArgumentError "Key: ... Can't parse serialized Example").
 *
 * Frames (TFRecord): u64 length | u32 masked_crc32c(length) | data | u32 masked_crc32c(data),
 * masked = ((c >> 15) | (c << 17)) + 0xa282ead8, c = CRC-32C.  Both CRCs are verified.
 *
 * Pipeline: a scanner thread walks epochs x files (each file mmapped once), checks the
 * frame headers, passes the frames through the shuffle buffer and groups them into batch
 * plans; `threads` decoders parse a plan's records in parallel straight into one of
 * `depth` ring batches; dlio_next copies the oldest ready batch into the caller's buffers
 * (row-major [batch, size] per feature, float32 or int64).  Batch order is deterministic
 * for a given seed (shuffle=0: file order).
 *
 * Errors: functions return < 0 and dlio_last_error(h) (or dlio_open_error() after a failed
 * open) gives the message.  One consumer thread per handle.
 */
#ifndef DLIO_H
#define DLIO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLIO_FLOAT 0
#define DLIO_INT64 1

typedef struct dlio_feature {
  const char* name;  /* feature key, e.g. "cate_feats" (data_loader.py:9-26)          */
  int32_t kind;      /* DLIO_FLOAT (tf.float32) or DLIO_INT64 (tf.int64)               */
  int32_t size;      /* FixedLenFeature shape [size]                                   */
} dlio_feature;

/* shuffle_buf <= 0: no shuffle (file order).  seed < 0: seeded from the OS (the
 * reference's shuffle is unseeded, data_loader.py:34).  repeat = epochs for 'train',
 * 1 otherwise (:38-39).  Returns NULL on error. */
void* dlio_open(const char* const* files, int32_t n_files, const dlio_feature* spec, int32_t n_feat,
                int32_t batch, int32_t repeat, int64_t shuffle_buf, int64_t seed, int32_t threads,
                int32_t depth);
/* Fills outs[j] (one buffer of batch * spec[j].size elements per feature).
 * Returns 1 = a batch was written, 0 = end of data (partial batch dropped), < 0 = error. */
int32_t dlio_next(void* h, void* const* outs);
/* Records decoded so far (including those of batches still in the ring). */
int64_t dlio_records(void* h);
const char* dlio_last_error(void* h);
const char* dlio_open_error(void);
void dlio_close(void* h);

/* One pickled load-style batch (utils/data_loader_load.py:128-136: a dict per batch whose values
 * are numpy arrays or lists of rows; models/wdl.py:296 unpickles one a step) decoded straight
 * into caller buffers: field j's dict value, rows x fields[j].size values, converted to float32
 * (DLIO_FLOAT) or int64 (DLIO_INT64), into outs[j] (room for cap_rows rows); *rows = the batch's
 * rows (every field the same).  No Python object is built and nothing named in the pickle is
 * constructed: protocols 3-5 of numpy arrays (numpy's reconstructors) and nested lists of
 * numbers only.  Returns 0 = decoded, 1 = a form this decoder does not take (a missing key,
 * another global, an object array, a shape that does not match: the caller unpickles in
 * Python), < 0 = malformed / bad arguments. */
int32_t dlio_unpickle_batch(const void* data, int64_t n, const dlio_feature* fields, int32_t n_fields,
                            int64_t cap_rows, void* const* outs, int64_t* rows);

/* CRC-32C (Castagnoli) of n bytes, and the TFRecord mask of it (SSE4.2 when present). */
uint32_t dlio_crc32c(const void* data, int64_t n);
uint32_t dlio_masked_crc32c(const void* data, int64_t n);

#ifdef __cplusplus
}
#endif
#endif /* DLIO_H */
