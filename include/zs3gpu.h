/*
 * zs3gpu.h — C ABI of the MI355X erasure-shard + bitrot-hash data path.
 *
 * Drop-in boundary for 0chain/zs3server's server-mode data path:
 * a cgo shim binds these entry points under the reference's
 *   - Erasure type           cmd/erasure-coding.go:35-150
 *   - bitrot hash factory    cmd/bitrot.go:47-64 (HighwayHash256S, key :37)
 *   - streaming bitrot I/O   cmd/bitrot-streaming.go:43-65, :142-189
 *   - encode / decode loops  cmd/erasure-encode.go:76-113, cmd/erasure-decode.go:206-332
 * replacing the arithmetic of github.com/klauspost/reedsolomon v1.11.8 and
 * github.com/minio/highwayhash v1.0.2.
 *
 * Conventions
 *   - Every function returns an int status: 0 = ZS3_OK, < 0 = one of the codes
 *     below, each mapped 1:1 to a reference error sentinel.  Size helpers return
 *     int64_t values exactly as the Go methods do.
 *   - Pointers named d_* are DEVICE pointers (HBM, from zs3_dev_alloc or any HIP
 *     allocation on the current device); h_* are host pointers.  The caller owns
 *     all memory it passes in; the library owns its codec tables and staging.
 *   - `stream` is a hipStream_t (NULL = the default stream of the current device).
 *     Device-batch calls are asynchronous on that stream; host calls are synchronous.
 *   - Shard layout inside one block ("stripe"): shard i is the S bytes at
 *     base + i*S, S = ShardSize = ceil(block_len / k) (erasure-coding.go:122).  This
 *     is exactly the reference's in-place Split layout in the bpool buffer
 *     (erasure-coding.go:81, cap = 2*blockSize, erasure-sets.go:383-387).
 *   - Thread-safety: codecs are immutable after creation except for internal
 *     caches guarded by a mutex; every entry point may be called concurrently.
 *     Host-pointer calls use per-OS-thread staging buffers and streams.
 */
#ifndef ZS3GPU_H
#define ZS3GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (reference sentinel each one maps to) ------------------ */
#define ZS3_OK                  0
#define ZS3_ERR_INV_SHARD_NUM  -1  /* reedsolomon.ErrInvShardNum  (erasure-coding.go:45)    */
#define ZS3_ERR_MAX_SHARD_NUM  -2  /* reedsolomon.ErrMaxShardNum  (erasure-coding.go:49)    */
#define ZS3_ERR_TOO_FEW_SHARDS -3  /* reedsolomon.ErrTooFewShards (erasure-utils.go:52)     */
#define ZS3_ERR_SHARD_NO_DATA  -4  /* reedsolomon.ErrShardNoData                            */
#define ZS3_ERR_SHARD_SIZE     -5  /* reedsolomon.ErrShardSize                              */
#define ZS3_ERR_SHORT_DATA     -6  /* reedsolomon.ErrShortData    (erasure-utils.go:58)     */
#define ZS3_ERR_FILE_CORRUPT   -7  /* errFileCorrupt (bitrot-streaming.go:185, bitrot.go:171) */
#define ZS3_ERR_INVALID_ARG    -8  /* errInvalidArgument / errUnexpected                    */
#define ZS3_ERR_DEVICE         -9  /* HIP runtime / kernel launch failure                   */
#define ZS3_ERR_NOMEM         -10  /* allocation failure                                    */
#define ZS3_ERR_SINGULAR      -11  /* internal: singular decode matrix (cannot happen for a valid pattern) */

const char* zs3_strerror(int code);
int zs3_version(void);                 /* (major << 16) | (minor << 8) | patch */

/* ---- device ---------------------------------------------------------------- */
int zs3_device_count(int* count);
int zs3_set_device(int device);        /* hipSetDevice for the calling OS thread */
int zs3_dev_alloc(void** d_ptr, size_t bytes);
int zs3_dev_free(void* d_ptr);
int zs3_host_alloc(void** h_ptr, size_t bytes);   /* pinned; backing for internal/bpool */
int zs3_host_free(void* h_ptr);                    /* a zs3_host_alloc pointer, else
                                                      ZS3_ERR_INVALID_ARG (nothing freed) */
int zs3_memcpy_h2d(void* d_dst, const void* h_src, size_t bytes, void* stream);
int zs3_memcpy_d2h(void* h_dst, const void* d_src, size_t bytes, void* stream);
int zs3_stream_sync(void* stream);

/* ---- codec: the Erasure value (erasure-coding.go:35-73) -------------------- */
typedef struct zs3_codec zs3_codec;

/* NewErasure (erasure-coding.go:42): k = dataBlocks, m = parityBlocks.
 * k <= 0 || m <= 0 -> ZS3_ERR_INV_SHARD_NUM; k + m > 256 -> ZS3_ERR_MAX_SHARD_NUM.
 * Builds (once) the klauspost systematic Vandermonde matrix for (k, m). */
int zs3_codec_new(int k, int m, int64_t block_size, zs3_codec** out);
void zs3_codec_free(zs3_codec* c);
int zs3_codec_matrix(const zs3_codec* c, uint8_t* h_out /* (k+m)*k bytes */);
/* The codec's dataBlocks, parityBlocks and blockSize (any pointer may be NULL). */
int zs3_codec_params(const zs3_codec* c, int* k, int* m, int64_t* block_size);

/* Size arithmetic, exact Go semantics (int64, -1 = unknown length). */
int64_t zs3_shard_size(const zs3_codec* c);                       /* Erasure.ShardSize      :122 */
int64_t zs3_shard_file_size(const zs3_codec* c, int64_t total);   /* Erasure.ShardFileSize  :127 */
int64_t zs3_shard_file_offset(const zs3_codec* c, int64_t start, int64_t length,
                              int64_t total);                     /* Erasure.ShardFileOffset :141 */
int64_t zs3_bitrot_shard_file_size(int64_t size, int64_t shard_size); /* bitrotShardFileSize bitrot.go:150 (HH256S) */

/* ---- device-resident batches ----------------------------------------------
 * A batch is n_blocks independent blocks of block_len bytes each (one 1 MiB
 * erasure block per object stripe, erasure-encode.go:83-111).  S = ceil(block_len/k).
 *
 * zs3_encode_batch: Split + Encode (+ HighwayHash-256 of every shard chunk) —
 *   EncodeData (erasure-coding.go:77) fused with streamingBitrotWriter.Write's
 *   h.Reset/h.Write/h.Sum (bitrot-streaming.go:47-49) for all k+m shards.
 *   data   : block b at d_data + b*data_stride, bytes [0, block_len); bytes up to
 *            k*S read as zero (Split padding) — they are not written.
 *   parity : block b parity row r at d_parity + b*parity_stride + r*S.  For the
 *            reference's in-place layout pass d_parity = d_data + k*S and
 *            parity_stride = data_stride.
 *   sums   : optional (NULL = encode only); block b shard i digest at
 *            d_sums + (b*(k+m) + i)*32, using the magic HH-256 key (bitrot.go:37).
 *   block_len == 0 is EncodeData's empty case: nothing is written (no shards, no
 *   sums, matching streamingBitrotWriter.Write's len(p)==0 no-op). */
int zs3_encode_batch(const zs3_codec* c, const uint8_t* d_data, int64_t data_stride,
                     int64_t block_len, int64_t n_blocks, uint8_t* d_parity,
                     int64_t parity_stride, uint8_t* d_sums, void* stream);

/* zs3_reconstruct_batch: ReconstructData (data_only != 0, DecodeDataBlocks
 *   erasure-coding.go:96) or Reconstruct (DecodeDataAndParityBlocks :113) on every
 *   block of a batch sharing one erasure pattern.  Block b shard i at
 *   d_shards + b*block_stride + i*shard_len.  present[i] != 0 marks shard i present
 *   (len != 0 in the Go [][]byte); missing rows are written in place.  Errors as
 *   reedsolomon: fewer than k present -> ZS3_ERR_TOO_FEW_SHARDS; nothing present ->
 *   ZS3_ERR_SHARD_NO_DATA; all needed present -> ZS3_OK with no work. */
int zs3_reconstruct_batch(const zs3_codec* c, uint8_t* d_shards, int64_t block_stride,
                          int64_t shard_len, int64_t n_blocks, const uint8_t* h_present,
                          int data_only, void* stream);

/* zs3_verify_reconstruct_batch: the GET / heal pass in one kernel.
 *   For every block: the k survivor shards the decode reads (the first k present,
 *   as ReconstructData picks them, erasure-coding.go:108) are HighwayHash-256'd and
 *   compared with their stored bitrot sums d_expect[b][i][32] (the 32-byte hash
 *   streamingBitrotReader.ReadAt checks, bitrot-streaming.go:171-186); then the missing
 *   shards (data only, or all with data_only == 0) are rebuilt in place from the same
 *   reads.  d_bad[b][i] (k+m int32 per block, zeroed first) = 1 where survivor i failed
 *   verification: that is the per-shard errFileCorrupt of erasure-decode.go:165-179,
 *   and the rebuilt shards of that block are then invalid — re-issue the block with
 *   shard i marked missing (parallelReader reads the next shard).  With d_sums_out
 *   != NULL the rebuilt shards are hashed too (heal: erasure-healing.go writes them
 *   through a new bitrot writer), digest at d_sums_out[b][i][32].  Nothing missing ->
 *   verify only.  Errors as zs3_reconstruct_batch. */
int zs3_verify_reconstruct_batch(const zs3_codec* c, uint8_t* d_shards, int64_t block_stride,
                                 int64_t shard_len, int64_t n_blocks, const uint8_t* h_present,
                                 int data_only, const uint8_t* d_expect, int32_t* d_bad,
                                 uint8_t* d_sums_out, void* stream);

/* HighwayHash-256 of n_msgs messages of msg_len bytes at d_msgs + i*msg_stride
 * (key = 32 bytes, NULL = the bitrot magic key).  Digest i at d_sums + 32*i. */
int zs3_hh256_batch(const uint8_t* h_key, const uint8_t* d_msgs, int64_t msg_stride,
                    int64_t msg_len, int64_t n_msgs, uint8_t* d_sums, void* stream);

/* Bitrot verify (streamingBitrotReader.ReadAt, bitrot-streaming.go:171-186): hash
 * each chunk and compare against d_want + 32*i; d_bad[i] = 1 where it differs
 * (the per-shard errFileCorrupt, never a whole-batch failure). */
int zs3_hh256_verify_batch(const uint8_t* h_key, const uint8_t* d_msgs, int64_t msg_stride,
                           int64_t msg_len, int64_t n_msgs, const uint8_t* d_want,
                           int32_t* d_bad, void* stream);

/* ---- per-block erasure patterns ---------------------------------------------
 * In the reference every block is decoded with its own shard set: parallelReader
 * nils a reader that failed or returned errFileCorrupt and reads the next shard
 * (cmd/erasure-decode.go:166-179), so the pattern can change from one block to the
 * next.  These take h_present as n_blocks rows of k+m bytes (row b = block b's
 * present flags, as zs3_reconstruct_batch's h_present) and serve every block with
 * its own (cached) decode plan; blocks sharing a pattern run in one launch.
 * h_status (optional, host, n_blocks int32) receives each block's status (the
 * reedsolomon error of its pattern, e.g. ZS3_ERR_TOO_FEW_SHARDS; failed blocks are
 * not touched).  Returns ZS3_OK when every block is OK, else the first block error;
 * the other blocks are still served.  Asynchronous on `stream` like the single-
 * pattern calls (the patterns are read before return). */
int zs3_reconstruct_batch_masks(const zs3_codec* c, uint8_t* d_shards, int64_t block_stride,
                                int64_t shard_len, int64_t n_blocks, const uint8_t* h_present,
                                int data_only, int32_t* h_status, void* stream);
int zs3_verify_reconstruct_batch_masks(const zs3_codec* c, uint8_t* d_shards, int64_t block_stride,
                                       int64_t shard_len, int64_t n_blocks, const uint8_t* h_present,
                                       int data_only, const uint8_t* d_expect, int32_t* d_bad,
                                       uint8_t* d_sums_out, int32_t* h_status, void* stream);

/* HighwayHash-256 of n_msgs messages of different lengths (SURVEY.md §8b
 * zs3_hh256_batch(key, msgs**, lens*, n)): message i is d_lens[i] bytes at
 * d_ptrs[i] (both DEVICE arrays; the pointers are device pointers).  A reader's last
 * chunk is shorter than the shard size (cmd/erasure-decode.go:112-114).  Digest i at
 * d_sums + 32*i. */
int zs3_hh256_batch_ragged(const uint8_t* h_key, const uint8_t* const* d_ptrs, const int64_t* d_lens,
                           int64_t n_msgs, uint8_t* d_sums, void* stream);

/* Deep-scan bitrotVerify for HighwayHash256S (cmd/bitrot.go:158-210, called by
 * xlStorage.VerifyFile cmd/xl-storage.go:2386-2404): n_files shard files resident on
 * the device in their on-disk layout [32-byte sum][chunk]* (file f at
 * d_files + f*file_stride, file_size bytes), the sums read in place.  want_size must
 * equal bitrotShardFileSize(part_size, shard_size), else ZS3_ERR_FILE_CORRUPT with
 * nothing launched (bitrot.go:159-162).  Chunks: ceil(part_size/shard_size), the last
 * one part_size - (chunks-1)*shard_size bytes.  d_bad (device, n_files*chunks int32)
 * receives 1 for every chunk whose HighwayHash-256 differs from its stored sum;
 * d_file_bad (optional device, n_files int32) receives 1 for every file with a bad
 * chunk (bitrotVerify's errFileCorrupt).  *chunks_out (optional) = chunks per file. */
int zs3_bitrot_verify_file_batch(const uint8_t* h_key, const uint8_t* d_files, int64_t file_stride,
                                 int64_t n_files, int64_t want_size, int64_t part_size, int64_t shard_size,
                                 int32_t* d_bad, int32_t* d_file_bad, int64_t* chunks_out, void* stream);

/* ---- PUT-stream object digests ------------------------------- */

/* S3 ETag of n_msgs objects: MD5 (RFC 1321, Go crypto/md5) of message i = d_msgs +
 * i*msg_stride, length d_lens[i] (device int64 array) or msg_len when d_lens is NULL.
 * Digest i (16 bytes) at d_out + 16*i.  Replaces etag.NewReader's md5.Write/Sum
 * (internal/etag/reader.go:106-144). */
int zs3_md5_batch(const uint8_t* d_msgs, int64_t msg_stride, int64_t msg_len, const int64_t* d_lens,
                  int64_t n_msgs, uint8_t* d_out, void* stream);

/* SHA-256 (FIPS 180-4, sha256-simd) of the same message layout; digest i (32 bytes,
 * big-endian) at d_out + 32*i.  Replaces hash.Reader's content SHA-256 checked at
 * EOF (internal/hash/reader.go:123-153). */
int zs3_sha256_batch(const uint8_t* d_msgs, int64_t msg_stride, int64_t msg_len, const int64_t* d_lens,
                     int64_t n_msgs, uint8_t* d_out, void* stream);

/* Independent messages of any lengths at any offsets in one launch (the parts of
 * multipart uploads: PutObjectPartHandler, cmd/object-handlers.go:2753, wraps each
 * part in hash.NewReader, :2919, for its ETag and content SHA-256,
 * internal/hash/reader.go:123-153): message i = d_base + d_offsets[i] with length
 * d_lens[i] (both device int64 arrays); digest i at d_out + 16*i (MD5) or 32*i
 * (SHA-256).  One lane per message: a launch takes as long as its longest message
 * (per-block latency roof in DESIGN.md §4), so group parts of similar size. */
int zs3_md5_parts(const uint8_t* d_base, const int64_t* d_offsets, const int64_t* d_lens, int64_t n_msgs,
                  uint8_t* d_out, void* stream);
int zs3_sha256_parts(const uint8_t* d_base, const int64_t* d_offsets, const int64_t* d_lens, int64_t n_msgs,
                     uint8_t* d_out, void* stream);

/* etag.Multipart (internal/etag/etag.go:211-226): h_etags holds n_etags ETags,
 * etag i at h_etags + offsets[i] with length lens[i] (16 = singlepart MD5; longer =
 * multipart "-N" or encrypted, both skipped as the reference skips them).  Writes
 * MD5(concatenated singlepart ETags) followed by "-<count>" to h_out (capacity >= 40)
 * and returns its length; returns 0 (nil ETag) when n_etags == 0.  The MD5 runs on
 * the device (zs3_md5_batch). */
int zs3_etag_multipart(const uint8_t* h_etags, const int64_t* offsets, const int64_t* lens, int64_t n_etags,
                       uint8_t* h_out);

/* Deterministic synthetic blocks (splitmix64 counter stream; identical to the
 * oracle's fill): block b gets object id obj0 + b. */
int zs3_fill_batch(uint8_t* d_out, int64_t stride, int64_t len, int64_t n_blocks,
                   uint64_t seed, uint64_t obj0, void* stream);

/* ---- host-pointer calls (synchronous; staged through pinned memory) ------- */

/* Erasure.EncodeData in place (erasure-coding.go:77-91 with the bpool buffer):
 * h_buf holds len data bytes and has capacity cap >= (k+m)*S.  On return bytes
 * [len, k*S) are zero (Split), parity row r is at h_buf + (k+r)*S, and if h_sums
 * is not NULL it receives the (k+m) HH-256 shard digests.  Returns S (>= 0) or an
 * error (cap too small -> ZS3_ERR_INVALID_ARG).  len == 0 returns 0. */
int64_t zs3_encode_data(const zs3_codec* c, uint8_t* h_buf, int64_t len, int64_t cap,
                        uint8_t* h_sums);

/* DecodeDataBlocks / DecodeDataAndParityBlocks on one host stripe of k+m rows of
 * shard_len bytes (missing rows may hold garbage; they are overwritten). */
int zs3_decode_data_blocks(const zs3_codec* c, uint8_t* h_shards, int64_t shard_len,
                           const uint8_t* h_present, int data_only);

/* HighwayHash-256 of one host message (key NULL = bitrot magic key). */
int zs3_hh256(const uint8_t* h_key, const uint8_t* h_msg, int64_t len, uint8_t* h_out32);

/* End-to-end streaming encode (BASELINE config 5): an object of
 * total_len host bytes (the PUT stream, erasure-encode.go:83-111 block loop) is cut
 * into block_size blocks; each block is Split + Encoded and all k+m shard chunks are
 * HighwayHash-256 summed on the device.  The pipeline double-buffers batches of
 * batch_blocks blocks: pageable -> pinned staging (host threads) -> H2D -> fused
 * kernel -> D2H, on separate streams.  Outputs (host):
 *   h_parity: block b parity row r at h_parity + b*m*S + r*S (S = ShardSize; the
 *             last partial block uses its own S' = ceil(len/k), rows still at m*S)
 *   h_sums:   block b shard i sum at h_sums + (b*(k+m) + i)*32
 * Data shards are the input bytes themselves (zero-padded for the last block), as
 * Split's in-place views.  Returns the number of blocks or an error. */
int64_t zs3_stream_encode(const zs3_codec* c, const uint8_t* h_src, int64_t total_len,
                          uint8_t* h_parity, uint8_t* h_sums, int64_t batch_blocks);

/* The same stream over several devices (BASELINE config 5: a multipart PUT on the 8
 * GPUs of a node): the full blocks are split into n_devices contiguous ranges
 * (zs3_split_range), one host thread + stream set + pinned slots per device, no data
 * exchanged between devices; the partial last block is encoded by the last device.
 * Outputs land at the same offsets as zs3_stream_encode's.  Pageable buffers are
 * staged through pinned memory by helper threads that overlap the GPU work. */
int64_t zs3_stream_encode_multi(const zs3_codec* c, const int* devices, int n_devices, const uint8_t* h_src,
                                int64_t total_len, uint8_t* h_parity, uint8_t* h_sums, int64_t batch_blocks);

/* Streamed GET / heal of one object (SURVEY.md §8f.1 / §8f.3 over a whole part): the
 * Erasure.Decode and Erasure.Heal block loops (erasure-decode.go:230-276, :287-332) in
 * device batches of batch_blocks blocks, pipelined (H2D of the next batch's survivor
 * rows || fused verify + rebuild (+ heal sums) || D2H of the previous batch's rebuilt
 * rows), so a lone large GET or heal does not pay a device round trip per block.
 *   h_stripes : the object's total_len bytes as ceil(total_len/blockSize) stripes, stripe b
 *               at h_stripes + b*(k+m)*S (S = ShardSize), row i at + i*S_b (S_b = S, the
 *               short last block its own ceil(len/k)); present rows hold the shard chunks
 *               the readers returned, missing rows anything.  Missing data rows (GET,
 *               data_only != 0) or all missing rows (heal) are rebuilt in place.
 *   h_present : n_blocks x (k+m) flags (a reader may drop out mid-object)
 *   h_expect  : n_blocks x (k+m) x 32 stored bitrot sums of the chunks (NULL: no verify);
 *               h_bad (n_blocks x (k+m) int32, optional) flags every survivor whose sum
 *               differs (errFileCorrupt: re-read that block with the shard dropped)
 *   h_sums_out: heal only (optional): n_blocks x (k+m) x 32, HighwayHash-256 of the rebuilt rows
 *   h_status  : optional n_blocks int32: each block's reedsolomon status
 * Pinned (zs3_host_alloc / hipHostMalloc) stripes move by DMA; pageable ones are staged by
 * helper threads.  Runs on the calling thread's device.  Returns the number of blocks, or
 * the first block's error (ZS3_ERR_TOO_FEW_SHARDS, ...) after serving every other block
 * (a failed block's missing rows are undefined). */
int64_t zs3_stream_decode(const zs3_codec* c, uint8_t* h_stripes, int64_t total_len, const uint8_t* h_present,
                          int data_only, const uint8_t* h_expect, int32_t* h_bad, uint8_t* h_sums_out,
                          int32_t* h_status, int64_t batch_blocks);

/* Range [lo, hi) of `total` units owned by `rank` of `world`: contiguous, near-equal,
 * the first total % world ranks one longer (the object / block split of the
 * multi-GPU paths). */
void zs3_split_range(int64_t total, int world, int rank, int64_t* lo, int64_t* hi);

/* ---- cross-request batching queue (SURVEY.md §8b Threading, §7 iv) ----------------
 * The reference calls EncodeData / DecodeDataBlocks once per 1 MiB block per request
 * (cmd/erasure-encode.go:83-111, cmd/erasure-decode.go:230-276); one block is far too
 * little work for one device round trip.  A queue gathers the blocks that concurrent
 * callers (OS threads: every goroutine inside cgo holds one) submit into device
 * batches on pinned staging slots; a batch's H2D copies run on its lane's H2D stream,
 * its kernels on its slot's stream and its D2H copies on the lane's D2H stream, so one
 * batch's results come back while the next batch goes in:
 *   - a block is copied into the queue's pinned staging by its submitting thread, or,
 *     when the caller's buffer lies inside a zs3_host_alloc allocation (the pinned
 *     bpool), holds a full-size block, opens its batch and no other batch of its lane
 *     is in flight (a lone caller), DMA'd from it directly (zero-copy: no host memcpy
 *     either way; parity / rebuilt rows are DMA'd straight back into it); under
 *     concurrency pinned blocks are staged like any other, which measured at least as
 *     fast;
 *   - a batch is launched when it is full, when fewer than slots-1 batches of its lane
 *     are in flight (batch while busy), when its oldest block has waited max_wait_us,
 *     or on flush; it is sealed — later blocks open the next batch — once it holds a
 *     third of its lane's live blocks on that device (submitted and not finished,
 *     callers waiting for a slot included; at least 8), so that with T synchronous
 *     callers three batches of ~T/3 overlap their copies and kernels.  A batch holds at most
 *     max(8, 64 MiB / blockSize) blocks (at most 512, and at most max_batch when set):
 *     the staging slots are sized to exactly that;
 *   - several devices (opts.devices): every device has its own slots, streams and
 *     threads; a block goes to the device with the fewest live blocks of its lane, and
 *     each device batches its own blocks (a node's GPUs and PCIe links share the load);
 *   - when the batch is done, zs3_req_wait copies its own block's results back into
 *     the caller's buffers on the calling thread; blocks nobody is waiting for are
 *     copied back by the queue's completion thread.
 * All entry points are thread-safe.  Every submitted request must be waited for
 * exactly once, before zs3_queue_free.  A submit may block while every staging slot
 * is in use, until a batch completes (never on other requests being waited for).
 * A queue serves ONE block size, its codec's: a block of exactly that length is full
 * (batched), a shorter one is an object's last block (launched on its own), a longer
 * one is ZS3_ERR_INVALID_ARG.  The reference builds NewErasure(k, m, blockSize) per
 * object with the object's own block size (1 MiB, or 10 MiB for legacy objects,
 * cmd/object-api-common.go:37-40), so a server keeps one codec + queue per
 * (k, m, blockSize). */
typedef struct zs3_queue zs3_queue;
typedef struct zs3_req zs3_req;
typedef struct {
    int device;       /* HIP device ordinal; -1 = the calling thread's current device
                         (ignored when n_devices > 0) */
    int max_batch;    /* upper bound on blocks per device batch (0 = the default:
                         max(8, 64 MiB / blockSize), at most 512).  Memory per lane in use,
                         per device: slots x batch x (k+m) x S of pinned host AND of device
                         memory (+ sums): RS(8+4) 1 MiB, 4 slots x 64 blocks = 384 MiB
                         each; the encode, GET and heal lanes are allocated on first use */
    int max_wait_us;  /* longest a block waits for its batch to fill (0 = 200) */
    int slots;        /* pinned staging slots (+ streams) per lane (0 = 4; at least 2) */
    const int* devices;  /* n_devices HIP ordinals to spread the blocks over (a node's
                            GPUs; repeats allowed); NULL / 0 = the one `device` */
    int n_devices;       /* 0..64 */
} zs3_queue_opts;

int zs3_queue_new(const zs3_codec* c, const zs3_queue_opts* opts /* NULL = defaults */, zs3_queue** out);
void zs3_queue_free(zs3_queue* q);

/* EncodeData (erasure-coding.go:77-91) of one block plus the k+m bitrot sums
 * (bitrot-streaming.go:47-49), exactly as zs3_encode_data: h_buf holds len data
 * bytes and has capacity cap >= (k+m)*S'; after zs3_req_wait bytes [len, k*S') are
 * zero, parity row r is at h_buf + (k+r)*S' and h_sums (optional) holds the (k+m)
 * digests.  len == 0 (the empty object) returns ZS3_OK and *req = NULL.  The buffers
 * must stay valid until zs3_req_wait returns. */
int zs3_queue_submit_encode(zs3_queue* q, uint8_t* h_buf, int64_t len, int64_t cap, uint8_t* h_sums,
                            zs3_req** req);

/* One block of k+m rows of shard_len bytes at h_shards (row i at h_shards +
 * i*shard_len; missing rows hold anything) with its own h_present[k+m].
 * data_only != 0: DecodeDataBlocks (missing data rows rebuilt); 0: Erasure.Heal's
 * DecodeDataAndParityBlocks (all missing rows rebuilt; h_sums_out, if given, receives
 * the HighwayHash-256 of every rebuilt row at i*32).  With h_expect ([k+m][32], the
 * sums stored in front of each chunk) the k survivors are verified in the same pass:
 * zs3_req_wait then returns ZS3_ERR_FILE_CORRUPT when any failed and h_bad (optional,
 * k+m int32) flags which (parallelReader drops that shard and reads the next,
 * erasure-decode.go:166-179; the rebuilt rows are invalid then).  zs3_req_wait
 * returns ZS3_OK or the block's reedsolomon error (e.g. ZS3_ERR_TOO_FEW_SHARDS). */
int zs3_queue_submit_decode(zs3_queue* q, uint8_t* h_shards, int64_t shard_len, const uint8_t* h_present,
                            int data_only, const uint8_t* h_expect, int32_t* h_bad, uint8_t* h_sums_out,
                            zs3_req** req);

/* Wait for one request, copy its results out, free the handle.  Returns S' for an
 * encode request, ZS3_OK for a decode request, or an error. */
int64_t zs3_req_wait(zs3_req* req);
int zs3_queue_flush(zs3_queue* q);   /* launch the open batches now */
int zs3_queue_stats(const zs3_queue* q, int64_t* batches, int64_t* blocks);
int64_t zs3_queue_zero_copy_blocks(const zs3_queue* q);  /* blocks DMA'd from / to pinned callers */
/* Per-device counters of a multi-device queue: index = position in opts.devices. */
int zs3_queue_device_stats(const zs3_queue* q, int index, int* device, int64_t* batches, int64_t* blocks);

/* Synchronous conveniences (submit + wait): what the cgo shim calls per block. */
int64_t zs3_queue_encode_data(zs3_queue* q, uint8_t* h_buf, int64_t len, int64_t cap, uint8_t* h_sums);
int zs3_queue_decode_data_blocks(zs3_queue* q, uint8_t* h_shards, int64_t shard_len, const uint8_t* h_present,
                                 int data_only, const uint8_t* h_expect, int32_t* h_bad);

/* Startup self-tests through the device path: erasureSelfTest
 * (erasure-coding.go:158-216, 60 (k, m) xxhash64 KATs + shard-0 rebuild) and
 * bitrotSelfTest (bitrot.go:218-249).  Returns ZS3_OK or ZS3_ERR_FILE_CORRUPT. */
int zs3_selftest(void);

/* Which kernel family served the last batch call on this thread (ZS3_PATH_*):
 * 0 = generic byte kernel, 1 = first-generation specialised (k, m) kernel,
 * 2 = warp-specialised kernel (k_ehx_ws / k_vr_ws), 3 = mixed-wave second-generation
 * encode (k_ehx), 4 = small-batch latency path (encode-only pass, then one chain per
 * quad straight from HBM: k_hash_lat); -1 = nothing launched. */
#define ZS3_PATH_NONE      -1
#define ZS3_PATH_GENERIC    0
#define ZS3_PATH_FIRSTGEN   1
#define ZS3_PATH_WS         2
#define ZS3_PATH_PIPE       3
#define ZS3_PATH_LATENCY    4
int zs3_last_path(void);

/* Every kernel family this thread's launches used since the previous call with reset != 0
 * (or since the thread started): bit (1u << ZS3_PATH_*) per family, plus
 * ZS3_KERNEL_VR_QUAD when the survivor-quad GET / heal kernel (k_vr_quad: RS(16+4) with four
 * rebuilt rows) served a batch.  Unlike zs3_last_path it survives the later launches of
 * one call (zs3_stream_decode's short last block), so a caller can check what every batch
 * of a streamed GET or heal ran on.  reset != 0 clears the set after reading it. */
#define ZS3_KERNEL_VR_QUAD (1u << 16)
uint32_t zs3_path_mask(int reset);

/* The stream drivers (zs3_stream_encode*, zs3_stream_decode) keep their pinned host and
 * device staging buffers for the next call (hipHostMalloc of a batch's slots costs more
 * than a large stream's own transfers).  At most `max_idle_bytes` stay idle per process
 * (default 6 GiB); this sets that cap, frees idle buffers past it at once (oldest first)
 * and returns the bytes freed.  zs3_pool_limit(0) releases every idle buffer. */
int64_t zs3_pool_limit(uint64_t max_idle_bytes);

#ifdef __cplusplus
}
#endif
#endif /* ZS3GPU_H */
