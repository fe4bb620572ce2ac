/*
 * hyrise_amd.h — C-ABI of the MI355X (gfx950) execution layer for Hyrise's TableScan / JoinHash / Aggregate
 * hot path.
 *
 * This is the drop-in boundary: the reference's operators keep their C++ surface
 * (AbstractOperator::_on_execute(), src/lib/operators/abstract_operator.hpp:70-172) and call into these entry
 * points for the per-chunk hot loops. Every entry point takes plain pointers and sizes, never throws, and returns
 * an hy_status (0 = success). Device buffers are caller-owned; every launch takes an explicit stream and a
 * caller-provided workspace whose size is queried first, so launches can be captured into hipGraphs.
 *
 * Which reference interface each entry point replaces is stated next to it (reference path:line).
 */
#ifndef HYRISE_AMD_H_
#define HYRISE_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int hy_status;
typedef void* hy_stream_t; /* hipStream_t */

enum {
  HY_OK = 0,
  HY_ERR_INVALID_ARGUMENT = 1,
  HY_ERR_DEVICE = 2,         /* a HIP runtime call failed; see hy_last_error_message() */
  HY_ERR_WORKSPACE = 3,      /* workspace too small */
  HY_ERR_ALIGNMENT = 4,      /* a device pointer is not 16-byte aligned */
  HY_ERR_UNSUPPORTED = 5,    /* type / mode not implemented on the device path */
  HY_ERR_CAPACITY = 6,       /* output capacity exceeded; *_required holds the needed size */
  HY_ERR_KERNEL = 7,         /* a kernel reported an internal failure (bounded spin expired) */
  HY_ERR_GROUP_BOUND = 8     /* hy_aggregate: more groups than params->group_bound allows; *n_groups holds the
                                group_bound to retry with (re-query the workspace size) */
};

/* RowID, identical layout to reference src/lib/types.hpp:97-131 ({ChunkID chunk_id; ChunkOffset chunk_offset;}). */
typedef struct hy_row_id {
  uint32_t chunk_id;
  uint32_t chunk_offset;
} hy_row_id;

/* Column data types (reference src/lib/all_type_variant.hpp data_types). */
enum { HY_TYPE_INT32 = 1, HY_TYPE_INT64 = 2, HY_TYPE_FLOAT = 3, HY_TYPE_DOUBLE = 4, HY_TYPE_STRING = 5 };

/* ---------------------------------------------------------------------------------------------------------------
 * Runtime
 * ------------------------------------------------------------------------------------------------------------- */
hy_status hy_get_device_count(int* count);
hy_status hy_set_device(int device);
hy_status hy_malloc(void** ptr, size_t bytes);
hy_status hy_free(void* ptr);
/* Stream-ordered allocation from the device's memory pool (kept across frees): for operator outputs that live as
 * long as their table. Freed memory is reused by later allocations ordered after the free on `stream`. */
hy_status hy_malloc_async(void** ptr, size_t bytes, hy_stream_t stream);
hy_status hy_free_async(void* ptr, hy_stream_t stream);
/* Frees `ptr` into the pool on `free_stream` after the work already enqueued on each of `wait_streams` (an event
 * recorded on each, waited for by `free_stream`): a buffer read by kernels of several non-blocking operator streams
 * returns to the pool only when all of them are done with it, and a later allocation on `free_stream` reuses it
 * without any cross-stream dependency. */
hy_status hy_free_async_after(void* ptr, hy_stream_t free_stream, const hy_stream_t* wait_streams, uint32_t n_wait);
/* The device pool's bytes held from the driver (reserved) and handed out (used). */
hy_status hy_pool_stats(uint64_t* reserved_bytes, uint64_t* used_bytes);
/* Free and total memory of the current device (hipMemGetInfo). */
hy_status hy_device_memory(uint64_t* free_bytes, uint64_t* total_bytes);
hy_status hy_memcpy_htod(void* dst, const void* src, size_t bytes, hy_stream_t stream);
hy_status hy_memcpy_dtoh(void* dst, const void* src, size_t bytes, hy_stream_t stream);
hy_status hy_memcpy_dtod(void* dst, const void* src, size_t bytes, hy_stream_t stream);
hy_status hy_memset(void* dst, int value, size_t bytes, hy_stream_t stream);
hy_status hy_stream_create(hy_stream_t* stream);
/* Waits for the stream's work, then destroys it. Streams handed to the entry points (which stage their host
 * descriptors through a per-thread pinned ring fenced by events on the caller's stream) are destroyed with this
 * function, which also drops those fences; an embedding that destroys such a stream itself first synchronises it. */
hy_status hy_stream_destroy(hy_stream_t stream);
hy_status hy_stream_synchronize(hy_stream_t stream);
/*
 * Per-kernel device timing (HIP events recorded around every launch on its stream; off by default).
 * collect() waits for the recorded launches and aggregates them per kernel name; get() reads one aggregate:
 * launches, summed device milliseconds, summed work units (rows or pairs the launches processed).
 */
hy_status hy_kernel_stats_enable(int enable);
hy_status hy_kernel_stats_reset(void);
hy_status hy_kernel_stats_collect(uint32_t* n_kernels);
hy_status hy_kernel_stats_get(uint32_t index, const char** name, uint64_t* launches, double* total_ms,
                              uint64_t* units);
/*
 * Debug: per-partition phase trace of the next hy_join_hash calls (NULL turns it off). When set, the first thread
 * of each partition's workgroup stores 5 wall-clock stamps (100 MHz device clock) at trace[5 * partition + i]:
 * entry, table built, probe counted, output offset known (look-back done), exit. Costs one scalar branch.
 */
hy_status hy_debug_set_join_trace(uint64_t* device_trace);
/*
 * Measured HBM roofline (the denominator of the bench's roofline fraction): HY_PROBE_READ streams
 * `bytes` from src (dst: a scratch buffer of 256 * 32 * 256 * 4 bytes, written only by a practically impossible
 * branch); HY_PROBE_COPY copies `bytes` from src to dst (2 * bytes of traffic). 16-byte nontemporal accesses, four in
 * flight per lane, a grid of up to 8192 workgroups. Launch only; time it with events on `stream`.
 */
enum { HY_PROBE_READ = 0, HY_PROBE_COPY = 1 };
hy_status hy_stream_bandwidth_probe(const void* src, void* dst, uint64_t bytes, int32_t mode, hy_stream_t stream);
/* Thread-local message of the last failing call. */
const char* hy_last_error_message(void);
/* Build identification ("gfx950 …"). */
const char* hy_build_info(void);

/* ---------------------------------------------------------------------------------------------------------------
 * Column chunk descriptors (device residency of the reference's per-chunk columns).
 *
 *   HY_COL_VALUE      ValueColumn<T>          reference src/lib/storage/value_column.hpp:15-73
 *                     data = T[size], nulls = uint8[size] (1 = NULL) or NULL when the column is not nullable
 *   HY_COL_DICT       DictionaryColumn<T>     reference src/lib/storage/dictionary_column.hpp:20-72
 *                     data = attribute vector (uint8/16/32 per vid_width, FixedSizeByteAligned,
 *                     reference vector_compression/fixed_size_byte_aligned/fixed_size_byte_aligned_compressor.cpp:21-43),
 *                     dictionary = T[dictionary_size] sorted unique, null_value_id = dictionary_size
 *                     (reference dictionary_column/dictionary_encoder.hpp:87)
 *
 *   HY_COL_STRING     ValueColumn<std::string> (same reference file): data = a packed string array (below) of
 *                     the chunk's size values, nulls as HY_COL_VALUE. A DICT chunk of strings keeps its attribute
 *                     vector in data and, when its strings are device-resident, a packed string array of its
 *                     dictionary_size entries in dictionary.
 *   packed string array of n strings: uint32 offsets[n + 1] (offsets[i] = byte start of string i, offsets[n] = total
 *                     bytes), then the bytes at (const char*)offsets + 4 * (n + 1) rounded up to 16. String i is
 *                     bytes[offsets[i], offsets[i + 1]) - std::string's value, compared byte-wise as unsigned char
 *                     (std::char_traits<char>::compare).
 *
 * All device pointers must be 16-byte aligned; buffers must be readable up to the next multiple of 16 bytes.
 * ------------------------------------------------------------------------------------------------------------- */
/*
 *   HY_COL_FOR        FrameOfReferenceColumn<int32/int64> (reference frame_of_reference_column.hpp, compressed form -
 *                     TableScans only: hy_table_scan / hy_table_scan_row_ids / hy_reference_scan): data = offsets
 *                     (vid_width 1 / 2 / 4 bytes, FixedSizeByteAligned), nulls = uint8 per row or NULL, dictionary =
 *                     block minima (value_type, one per 2048 rows); row value = minima[row / 2048] + offset[row]
 *   HY_COL_RLE        RunLengthColumn<T> (reference run_length_column.hpp, compressed form - TableScans only): data =
 *                     run values (T[dictionary_size]), nulls = uint8 per run or NULL, dictionary = end_positions
 *                     (uint32[dictionary_size], the last row of each run, ascending), dictionary_size = runs.
 *                     RunLengthColumn<std::string> (string scans only): data = a packed string array (below) of
 *                     the runs' values, the rest as above; the predicate is evaluated once per run.
 *   FixedStringDictionaryColumn (reference fixed_string_dictionary_column.hpp) is passed as HY_COL_DICT: its
 *                     fixed-width entries decoded up to their first '\0', as a packed string array in dictionary.
 * The other entry points (joins, aggregates, projections, column compares) read these chunks as HY_COL_VALUE mirrors
 * (hy_decode_run_length / hy_decode_frame_of_reference) and reject HY_COL_FOR / HY_COL_RLE with HY_ERR_UNSUPPORTED.
 */
enum { HY_COL_VALUE = 0, HY_COL_DICT = 1, HY_COL_STRING = 2, HY_COL_FOR = 3, HY_COL_RLE = 4 };

typedef struct hy_column_chunk {
  const void* data;          /* values (VALUE) or attribute vector (DICT) */
  const uint8_t* nulls;      /* VALUE: null flags or NULL; DICT: unused */
  const void* dictionary;    /* DICT: sorted dictionary (device) */
  uint32_t size;             /* rows in this chunk */
  uint32_t dictionary_size;  /* DICT: number of dictionary entries (== null value id) */
  int32_t kind;              /* HY_COL_VALUE / HY_COL_DICT */
  int32_t vid_width;         /* DICT: 1, 2 or 4 bytes */
} hy_column_chunk;

/* ---------------------------------------------------------------------------------------------------------------
 * TableScan (single column vs constant)
 *
 * Replaces the per-chunk hot loop BaseTableScanImpl::_unary_scan_with_value / _unary_scan
 * (reference src/lib/operators/table_scan/base_table_scan_impl.hpp:33-63) as driven by
 * SingleColumnTableScanImpl::handle_column (single_column_table_scan_impl.cpp:38-142) for all chunks of a table
 * in ONE launch. The dictionary rewrite (search value id via lower/upper_bound and the all/none early-outs,
 * single_column_table_scan_impl.cpp:145-205) is host work per chunk and arrives here as (op, search_vid).
 *
 * Output is order-preserving: for chunk c the matching chunk offsets are written ascending at
 * out_offsets + out_begin[c] and counts[c] receives the number of matches, exactly the PosList the reference
 * builds for that chunk ({c, offset} for each match).
 * ------------------------------------------------------------------------------------------------------------- */
enum {
  HY_OP_EQ = 0, /* ==  */
  HY_OP_NE = 1, /* !=  */
  HY_OP_LT = 2, /* <   */
  HY_OP_LE = 3, /* <=  */
  HY_OP_GT = 4, /* >   */
  HY_OP_GE = 5, /* >=  */
  HY_OP_ALL = 6, /* every non-NULL row (dictionary "matches all" early-out) */
  HY_OP_NONE = 7, /* no row (dictionary "matches none" early-out) */
  /* IS NULL / IS NOT NULL (reference IsNullTableScanImpl, is_null_table_scan_impl.cpp:20-117): no constant, no
   * dictionary rewrite; DICT rows are NULL iff vid == dictionary_size, VALUE rows iff their null flag is set.
   * Supported by hy_table_scan / hy_table_scan_row_ids / hy_reference_scan; the fused scan filters of
   * hy_scan_join_hash and hy_aggregate reject HY_OP_IS_NULL with HY_ERR_UNSUPPORTED. */
  HY_OP_IS_NULL = 8,
  HY_OP_IS_NOT_NULL = 9, /* every non-NULL row (same rows as HY_OP_ALL) */
  /* DICT chunks only: rows whose value id v is set in vid_set (bit v % 32 of word v / 32). LIKE / NOT LIKE: the host
   * evaluates the pattern once per dictionary entry (LikeTableScanImpl::_find_matches_in_dictionary,
   * like_table_scan_impl.cpp:48-83, 102-120) and the device scans the attribute vector against that set. Scans only
   * (the fused filters of hy_scan_join_hash / hy_aggregate reject it). */
  HY_OP_VID_SET = 10,
  /* STRING chunks only (hy_string_table_scan / hy_string_reference_scan): the row's value matches / does not match
   * the LIKE pattern of the call's hy_string_predicate (LikeTableScanImpl on a value column,
   * like_table_scan_impl.cpp:22-31, 86-97, with the reference's LikeMatcher, like_matcher.cpp:9-118). */
  HY_OP_LIKE = 11,
  HY_OP_NOT_LIKE = 12
};

typedef struct hy_scan_chunk {
  hy_column_chunk column;
  int32_t op;            /* HY_OP_*; for DICT chunks compared against search_vid */
  uint32_t search_vid;   /* DICT: search value id (host-computed, reference _get_search_value_id) */
  uint64_t out_begin;    /* first output slot of this chunk (capacity = column.size) */
  const uint32_t* vid_set; /* HY_OP_VID_SET: device bitmap over the chunk's value ids, else unused (NULL) */
} hy_scan_chunk;

/* Workspace bytes for a scan over chunks with the given sizes. */
hy_status hy_table_scan_workspace_size(const uint32_t* chunk_sizes, uint32_t n_chunks, size_t* bytes);

/*
 * value_type: HY_TYPE_* of VALUE chunks (ignored for DICT chunks). constant: host pointer to one value of
 * value_type (the type_cast<T>(right_value) of the reference). chunks: HOST array. out_offsets and counts: device.
 */
hy_status hy_table_scan(const hy_scan_chunk* chunks, uint32_t n_chunks, int32_t value_type, const void* constant,
                        uint32_t* out_offsets, uint32_t* counts, void* workspace, size_t workspace_bytes,
                        hy_stream_t stream);

/*
 * Same scan, writing reference RowIDs {chunk_ids[c], offset} (8 B each) at out_rows + out_begin[c] — the PosList
 * of the output chunk as the reference stores it (used by fused Scan -> Join pipelines). chunk_ids: HOST array.
 */
hy_status hy_table_scan_row_ids(const hy_scan_chunk* chunks, uint32_t n_chunks, int32_t value_type,
                                const void* constant, const uint32_t* chunk_ids, hy_row_id* out_rows, uint32_t* counts,
                                void* workspace, size_t workspace_bytes, hy_stream_t stream);

/*
 * Matches per chunk of a scan over DICT chunks, counted only (no output): counts[c] (device) = the rows of chunk c
 * that hy_table_scan would emit. chunks: HOST array (one id width over the non-empty chunks, no IS NULL); workspace:
 * n_chunks * sizeof(hy_scan_chunk) bytes. The row count a TableScan's consumer needs before the scan itself runs
 * fused into that consumer (a JoinHash's swap rule compares its inputs' row counts, join_hash.cpp:55-76).
 */
hy_status hy_table_scan_count(const hy_scan_chunk* chunks, uint32_t n_chunks, uint32_t* counts, void* workspace,
                              size_t workspace_bytes, hy_stream_t stream);

/*
 * Scan over a ReferenceColumn (reference BaseSingleColumnTableScanImpl::handle_column(const ReferenceColumn&),
 * base_single_column_table_scan_impl.cpp:36-60): for each position i of pos_list (device RowIDs) whose RowID is
 * not NULL, the referenced value is read from referenced_chunks[row.chunk_id] and compared. Positions of matches
 * are written ascending to out_positions; *count (device) receives the number of matches. Per referenced chunk
 * the predicate is given by ref_scan[row.chunk_id] (op + search_vid, because dictionaries differ per chunk).
 * Group ordering of the reference's unordered_map over referenced chunks is applied by the caller
 * (hy_reference_scan_order).
 */
hy_status hy_reference_scan_workspace_size(uint64_t pos_list_size, size_t* bytes);
hy_status hy_reference_scan(const hy_row_id* pos_list, uint64_t pos_list_size, const hy_scan_chunk* referenced_chunks,
                            uint32_t n_referenced_chunks, int32_t value_type, const void* constant,
                            uint32_t* out_positions, uint64_t* count, void* workspace, size_t workspace_bytes,
                            hy_stream_t stream);

/*
 * Positions i of pos_list whose RowID is NULL (chunk_offset == INVALID_CHUNK_OFFSET), ascending, to out_positions;
 * *count (device) receives their number. An IS NULL scan over a ReferenceColumn appends these after the matches of
 * the referenced columns (reference IsNullTableScanImpl::handle_column(const ReferenceColumn&),
 * is_null_table_scan_impl.cpp:20-33). Workspace as hy_reference_scan_workspace_size(pos_list_size).
 */
hy_status hy_pos_list_null_positions(const hy_row_id* pos_list, uint64_t pos_list_size, uint32_t* out_positions,
                                     uint64_t* count, void* workspace, size_t workspace_bytes, hy_stream_t stream);

/*
 * out[i] = pos_list[positions[i]] for i < n (device gather; builds the filtered PosList of a reference-input
 * scan, reference table_scan.cpp:124-134, and the dereference of write_output_columns, join_hash.cpp:584-592).
 */
hy_status hy_gather_row_ids(const hy_row_id* pos_list, const uint32_t* positions, uint64_t n, hy_row_id* out,
                            hy_stream_t stream);

/*
 * Reference-input TableScan over a PosList referencing several chunks, in the reference's output order: the
 * reference splits the PosList by referenced chunk into a std::unordered_map (split_pos_list_by_chunk_id,
 * chunk_offset_mapping.cpp:5-21) and emits the matches group by group in the map's iteration order, positions
 * ascending inside a group (base_single_column_table_scan_impl.cpp:36-60). Given the ascending match positions of
 * ONE hy_reference_scan over all chunks, writes them to out_positions ordered by (chunk_rank[referenced chunk id],
 * position): chunk_rank (device, n_chunks entries, values < n_ranks) is the group order the host replays
 * (std::unordered_map iteration order). One launch and one stable radix sort instead of one scan per group.
 */
hy_status hy_reference_scan_order_workspace_size(uint64_t n, uint32_t n_ranks, size_t* bytes);
hy_status hy_reference_scan_order(const hy_row_id* pos_list, const uint32_t* positions, uint64_t n,
                                  const uint32_t* chunk_rank, uint32_t n_chunks, uint32_t n_ranks,
                                  uint32_t* out_positions, void* workspace, size_t workspace_bytes,
                                  hy_stream_t stream);

/*
 * first_seen[c] = smallest position i with pos_list[i].chunk_id == c (NULL RowIDs skipped), ~0 if none, for
 * c < n_chunks. Gives the order in which split_pos_list_by_chunk_id (reference
 * src/lib/storage/column_iterables/chunk_offset_mapping.cpp:5-21) first inserts each referenced chunk.
 */
hy_status hy_pos_list_chunk_first_seen(const hy_row_id* pos_list, uint64_t n, uint32_t n_chunks, uint64_t* first_seen,
                                       hy_stream_t stream);

/* out[i] = {chunk_id, offsets[i]} — expands a single-chunk offset list into reference RowIDs. */
hy_status hy_expand_row_ids(uint32_t chunk_id, const uint32_t* offsets, uint64_t n, hy_row_id* out,
                            hy_stream_t stream);
/* The same for the offset lists of n_chunks chunks in one launch (a fused TableScan's output of hy_scan_join_hash):
 * out[i] = {chunk_ids[c], offsets[i]} for i in [chunk_begin[c], chunk_begin[c + 1]). All device arrays; chunk_ids
 * NULL means chunk id c. Replaces the per-chunk PosList materialisation of table_scan.cpp:87-99 for a scan whose
 * matches its consumer's join computed. */
hy_status hy_expand_chunk_row_ids(const uint32_t* offsets, const uint64_t* chunk_begin, const uint32_t* chunk_ids,
                                  uint32_t n_chunks, hy_row_id* out, hy_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------------
 * String scans (std::string columns; reference SingleColumnTableScanImpl / LikeTableScanImpl / IsNullTableScanImpl
 * on a ValueColumn<std::string>, single_column_table_scan_impl.cpp:38-85, like_table_scan_impl.cpp:22-31, 86-97,
 * is_null_table_scan_impl.cpp:35-117)
 *
 * Chunks are HY_COL_STRING (compared with pred->value: HY_OP_EQ..HY_OP_GE as std::string::compare, unsigned bytes then
 * length; HY_OP_LIKE / HY_OP_NOT_LIKE against pred->pattern; IS [NOT] NULL, ALL, NONE), HY_COL_RLE of strings (the
 * same predicate on each run's value, spread to the run's rows) or HY_COL_DICT (op + search_vid or HY_OP_VID_SET exactly
 * as hy_table_scan: the host's dictionary rewrite). A table may mix them (an unencoded chunk beside dictionary and
 * run-length chunks). NULL rows never match a comparison or LIKE.
 * pattern_regex: 0 for the reference's simple patterns (LikeMatcher::pattern_string_to_pattern_tokens gives
 * StartsWith / EndsWith / Contains / MultipleContains: '%' and '_' match any byte), 1 for every other pattern (the
 * reference's std::regex path, like_matcher.cpp:27-52: '%' and '_' match any byte but '\n' / '\r'; '[...]' is a
 * character class of the bytes inside, '%' inside one meaning '.' and '*', '_' meaning '.'). At most 63 pattern
 * positions; "x-y" ranges of plain bytes; anything else the regex would reject -> HY_ERR_UNSUPPORTED.
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct hy_string_predicate {
  const char* value;      /* HOST: the constant (comparison ops), value_len bytes */
  uint32_t value_len;
  int32_t pattern_regex;  /* see above */
  const char* pattern;    /* HOST: the LIKE pattern (HY_OP_LIKE / HY_OP_NOT_LIKE), pattern_len bytes */
  uint32_t pattern_len;
  uint32_t reserved;
} hy_string_predicate;

/* Data input: the matches of all chunks as RowIDs {chunk_ids[c], offset}, chunk-major, offsets ascending, at out_rows
 * (device, capacity = rows); counts[c] (device) per chunk, *n_out (device) in total. chunks / chunk_ids: HOST arrays
 * (out_begin unused). */
hy_status hy_string_table_scan_workspace_size(const hy_scan_chunk* chunks, uint32_t n_chunks,
                                              const hy_string_predicate* pred, size_t* bytes);
hy_status hy_string_table_scan(const hy_scan_chunk* chunks, uint32_t n_chunks, const hy_string_predicate* pred,
                               const uint32_t* chunk_ids, hy_row_id* out_rows, uint32_t* counts, uint64_t* n_out,
                               void* workspace, size_t workspace_bytes, hy_stream_t stream);
/* Reference input: as hy_reference_scan (positions of matching pos_list entries, ascending; NULL RowIDs never match). */
hy_status hy_string_reference_scan_workspace_size(uint64_t pos_list_size, uint32_t n_referenced,
                                                  const hy_string_predicate* pred, size_t* bytes);
hy_status hy_string_reference_scan(const hy_row_id* pos_list, uint64_t pos_list_size,
                                   const hy_scan_chunk* referenced_chunks, uint32_t n_referenced_chunks,
                                   const hy_string_predicate* pred, uint32_t* out_positions, uint64_t* count,
                                   void* workspace, size_t workspace_bytes, hy_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Validate (MVCC visibility, reference src/lib/operators/validate.cpp:14-95)
 *
 * Row r of a chunk with MVCC columns is visible to transaction our_tid under snapshot_commit_id iff
 *   snapshot_commit_id < end_cids[r] && ((snapshot_commit_id >= begin_cids[r]) != (tids[r] == our_tid)).
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct hy_mvcc_chunk {
  const uint32_t* tids;        /* device: TransactionID per row (0 unless locked), reference mvcc_columns.hpp:22 */
  const uint32_t* begin_cids;  /* device: CommitID of the insert */
  const uint32_t* end_cids;    /* device: CommitID of the delete (MAX_COMMIT_ID = 2^32-2 if none) */
  uint32_t size;               /* rows */
  uint32_t reserved;
} hy_mvcc_chunk;

/* n_rows: total rows of the chunks (hy_validate) or the PosList length (hy_validate_pos_list); n_chunks: chunks /
 * referenced chunks. */
hy_status hy_validate_workspace_size(uint64_t n_rows, uint32_t n_chunks, size_t* bytes);
/* Data-table input: visible rows as RowIDs {chunk_ids[c], offset}, chunk-major, offsets ascending, at out_rows;
 * counts[c] (device) per chunk, *n_out (device) in total. chunks / chunk_ids: HOST arrays. */
hy_status hy_validate(const hy_mvcc_chunk* chunks, uint32_t n_chunks, const uint32_t* chunk_ids, uint32_t our_tid,
                      uint32_t snapshot_commit_id, hy_row_id* out_rows, uint32_t* counts, uint64_t* n_out,
                      void* workspace, size_t workspace_bytes, hy_stream_t stream);
/* Reference input: the RowIDs of pos_list (into the referenced table, whose chunks' MVCC columns are
 * referenced_chunks, HOST array indexed by chunk id) that are visible, in PosList order, at out_rows. NULL RowIDs are
 * dropped. */
hy_status hy_validate_pos_list(const hy_row_id* pos_list, uint64_t pos_list_size,
                               const hy_mvcc_chunk* referenced_chunks, uint32_t n_referenced, uint32_t our_tid,
                               uint32_t snapshot_commit_id, hy_row_id* out_rows, uint64_t* n_out, void* workspace,
                               size_t workspace_bytes, hy_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Encoded chunks -> value mirrors in HBM (all pointers device)
 * ------------------------------------------------------------------------------------------------------------- */
/* SIMD-BP128 attribute vector (reference vector_compression/simd_bp128/, simd_bp128_decompressor.cpp) -> the
 * FixedSizeByteAligned ids (out_width 1 / 2 / 4 bytes per id). words: the 16-byte words of the packing (per meta block
 * of 2048 ids a header word of 16 bit widths, then each 128-id block's `width` words, id j of a block in 32-bit lane
 * j % 4 at bit (j / 4) * width of that lane's stream); meta_offsets[m]: index (in 16-byte words) of meta block m's
 * header, ceil(n_rows / 2048) entries. */
hy_status hy_decode_simd_bp128(const void* words, const uint32_t* meta_offsets, uint32_t n_rows, int32_t out_width,
                               void* out, hy_stream_t stream);
/* RunLengthColumn (reference storage/run_length_column.hpp, run_length_column.cpp:24-36): row i takes the value and
 * NULL flag of the first run r with end_positions[r] >= i. value_bytes 4 or 8; out_nulls may be NULL. */
hy_status hy_decode_run_length(const void* values, const uint8_t* run_nulls, const uint32_t* end_positions,
                               uint32_t n_runs, uint32_t value_bytes, uint32_t n_rows, void* out_values,
                               uint8_t* out_nulls, hy_stream_t stream);
/* FrameOfReferenceColumn (reference frame_of_reference_column.cpp:25-37): value = block_minima[i / 2048] + offset[i],
 * offsets FixedSizeByteAligned of offset_width 1/2/4 bytes; value_type HY_TYPE_INT32 / HY_TYPE_INT64. (NULL flags
 * are uploaded as they are.) */
hy_status hy_decode_frame_of_reference(const void* block_minima, int32_t value_type, const void* offsets,
                                       int32_t offset_width, uint32_t n_rows, void* out_values, hy_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Hashing (reference src/lib/utils/murmur_hash.cpp:21-75, seed 17 from join_hash.cpp:680)
 * ------------------------------------------------------------------------------------------------------------- */
/* out[i] = murmur_hash2(&keys[i], key_bytes, seed); key_bytes 4 or 8. */
/* MurmurHash2 of a byte string (murmur_hash.cpp:21-73), host function: the hash of a std::string key. */
uint32_t hy_murmur2_bytes(const void* bytes, uint32_t len, uint32_t seed);
hy_status hy_murmur2(const void* keys, uint64_t n, uint32_t key_bytes, uint32_t seed, uint32_t* out,
                     hy_stream_t stream);
/* Radix bits of JoinHashImpl's constructor (join_hash.cpp:640-668) for a build side of build_rows rows. */
uint32_t hy_join_radix_bits(uint64_t build_rows, uint32_t key_bytes);

/* ---------------------------------------------------------------------------------------------------------------
 * JoinHash (equi-join, radix partitioned)
 *
 * Replaces JoinHashImpl::_on_execute's materialize_input / partition_radix_parallel / build / probe
 * (reference src/lib/operators/join_hash.cpp:203-527). One side of the join ("build" / "probe" after the
 * reference's swap rule, join_hash.cpp:55-76) is described by a list of chunks. A chunk is either a column chunk
 * of a data table, or — for a reference table — a device PosList into referenced column chunks.
 *
 * Output reproduces the reference exactly: one output chunk per radix partition p (ascending) with at least one
 * emitted pair; inside a partition, probe rows in (chunk, offset) order and for each probe row its build matches
 * in build (chunk, offset) order. partition_counts[p] = pairs of partition p, written at
 * [partition_begin[p], partition_begin[p] + partition_counts[p]) of out_build / out_probe.
 * Rows are emitted as RowIDs of the side's input table: (input chunk id, offset in that chunk / in the
 * ReferenceColumn), like the reference before write_output_columns; NULL_ROW_ID for the outer side of a
 * Left/Right join without match. Semi/Anti write only out_probe.
 * ------------------------------------------------------------------------------------------------------------- */
enum { HY_JOIN_INNER = 0, HY_JOIN_LEFT = 1, HY_JOIN_RIGHT = 2, HY_JOIN_SEMI = 5, HY_JOIN_ANTI = 6 };

#define HY_MIXED_CHUNKS 0xFFFFFFFFu

typedef struct hy_join_chunk {
  hy_column_chunk column;      /* data-table chunk (pos_list == NULL) */
  const hy_row_id* pos_list;   /* reference-table chunk: device PosList of this chunk, or NULL */
  uint32_t size;               /* rows of this chunk (== column.size or PosList length) */
  uint32_t chunk_id;           /* chunk id of this chunk in its table */
  uint32_t single_chunk;       /* reference chunk: index in the side's `referenced` array of the only referenced
                                  chunk when every non-NULL RowID of pos_list points into it (e.g. a TableScan output
                                  over a data table), else HY_MIXED_CHUNKS. Zero-initialised descriptors must set it. */
  uint32_t referenced_offset;  /* reference chunk: index in `referenced` of the first chunk of the table its PosList
                                  references - a column whose chunks reference several tables lists those tables'
                                  chunks one table after the other (RowID chunk_id c then reads referenced[
                                  referenced_offset + c - referenced_chunk_base]); 0 with one referenced table */
} hy_join_chunk;

typedef struct hy_join_side {
  const hy_join_chunk* chunks;            /* HOST array, one per chunk of the side's table */
  uint32_t n_chunks;
  int32_t value_type;                     /* HY_TYPE_* of the join column */
  const hy_column_chunk* referenced;      /* HOST array: column chunks of the referenced table (reference sides) */
  uint32_t n_referenced;
  /* reference sides only: 1 = emit RowIDs of the referenced table (fused write_output_columns dereference, valid
   * when every output column of this side shares the join column's PosLists); 0 = emit RowIDs of the side's own
   * table, to be dereferenced per PosList group with hy_dereference_row_ids. */
  int32_t fuse_dereference;
  /* reference sides: RowIDs in the PosLists name referenced chunk referenced_chunk_base + i for referenced[i] (a
   * rank of the distributed join holds a range of a table's chunks under their global ids); 0 otherwise */
  uint32_t referenced_chunk_base;
} hy_join_side;

/*
 * Column-vs-column TableScan (reference ColumnComparisonTableScanImpl::scan_chunk,
 * column_comparison_table_scan_impl.cpp:23-84 + BaseTableScanImpl::_binary_scan, base_table_scan_impl.hpp:64-76):
 * for every chunk c of the two sides (same chunk count and sizes; both data chunks or both PosLists, the reference's
 * "Invalid column combination" otherwise), row i matches iff neither value is NULL (a NULL RowID reads as NULL) and
 * `left OP right` holds with op in HY_OP_EQ..HY_OP_GE under C++'s usual arithmetic conversions of the two
 * HY_TYPE_* value types. Matches are written chunk-major, offsets ascending: either as RowIDs
 * {left.chunks[c].chunk_id, i} (out_rows) or as chunk offsets (out_offsets) - exactly one of the two. counts[c]
 * (device, n_chunks) receives the matches of chunk c, *n_out (device) their total; chunk c's matches start at the sum
 * of counts of the chunks before it. Sides are hy_join_side descriptors (value_type, chunks, referenced chunks);
 * fuse_dereference is ignored. String columns: both value types HY_TYPE_STRING (a string and a numeric column:
 * HY_ERR_INVALID_ARGUMENT), chunks HY_COL_STRING or HY_COL_DICT with a packed string dictionary, compared as
 * std::string's operators (unsigned bytes, then length).
 */
hy_status hy_column_compare_scan_workspace_size(const hy_join_side* left, const hy_join_side* right, int32_t out_rows,
                                                size_t* bytes);
hy_status hy_column_compare_scan(const hy_join_side* left, const hy_join_side* right, int32_t op,
                                 hy_row_id* out_rows, uint32_t* out_offsets, uint32_t* counts, uint64_t* n_out,
                                 void* workspace, size_t workspace_bytes, hy_stream_t stream);


typedef struct hy_join_params {
  int32_t mode;           /* HY_JOIN_* */
  int32_t hashed_type;    /* HY_TYPE_* of JoinHashTraits<L,R>::HashType (hash_traits.hpp:9-42) */
  uint32_t radix_bits;    /* normally hy_join_radix_bits(build rows) */
  uint32_t seed;          /* 17 */
  /* String join keys (JoinHashTraits HashType std::string, hash_traits.hpp:36-41): NULL, or a device table of
   * murmur2 hashes of distinct strings (hy_murmur2_bytes): the sides' int32 values are then ids into it (equal
   * strings, equal ids) and a row's partition follows key_hash[id] - the reference's hash of the string. Single-GPU
   * joins only (hy_join_hash / hy_scan_join_hash). */
  const uint32_t* key_hash;
} hy_join_params;

typedef struct hy_join_result {
  uint64_t total_pairs;        /* written by hy_join_hash */
  uint64_t capacity_required;  /* set when HY_ERR_CAPACITY is returned */
} hy_join_result;

hy_status hy_join_hash_workspace_size(const hy_join_side* build, const hy_join_side* probe,
                                      const hy_join_params* params, size_t* bytes);
/*
 * out_build / out_probe: device RowID arrays of capacity out_capacity pairs.
 * partition_begin / partition_counts: device arrays of 2^radix_bits uint64 / uint32.
 */
hy_status hy_join_hash(const hy_join_side* build, const hy_join_side* probe, const hy_join_params* params,
                       hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                       uint32_t* partition_counts, hy_join_result* result, void* workspace, size_t workspace_bytes,
                       hy_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Fused TableScan -> JoinHash.
 *
 * The plan TableScan(T, col OP value) -> JoinHash(..., <scan output>, ...) (reference lqp_translator.cpp:169 / :330,
 * table_scan.cpp:78-164 feeding join_hash.cpp:49-858) executed as one device pipeline: the scan predicate of a join
 * side is evaluated inside the join's first radix pass, which reads the data table's chunks directly, so the scan's
 * output is never re-read to gather the join column. The result is exactly that of the two operators:
 *   - out_offsets / out_chunk_begin: the TableScan's output, chunk by chunk - the matching chunk offsets of chunk c
 *     (ascending, base_table_scan_impl.hpp:50-63) at out_offsets[out_chunk_begin[c], out_chunk_begin[c + 1]); chunk c
 *     of the side is an output chunk of the scan iff it has a match (table_scan.cpp:99), and its PosList is
 *     {chunk_id of side chunk c, offset} for each offset;
 *   - the join output (as hy_join_hash) with the filtered side's RowIDs naming rows of the DATA table, i.e. the
 *     JoinHash output already dereferenced through the scan's PosLists (write_output_columns, join_hash.cpp:584-592).
 * The side must be a data table (no PosLists); its chunks and the predicate chunks correspond one to one (the
 * predicate column is another column of the same table). Either filter may be NULL (no scan on that side);
 * out_offsets / out_chunk_begin may be NULL when only the join output is wanted.
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct hy_join_filter {
  const hy_scan_chunk* chunks;  /* HOST array, one per chunk of the side: the predicate column's chunk (op, search_vid
                                   from the host dictionary rewrite exactly as for hy_table_scan; out_begin unused) */
  int32_t value_type;           /* HY_TYPE_* of VALUE predicate chunks */
  const void* constant;         /* HOST pointer to the constant of VALUE predicate chunks (type_cast<T>(value)) */
  uint32_t* out_offsets;        /* device, capacity = side rows, or NULL */
  uint64_t* out_chunk_begin;    /* device, n_chunks + 1 entries, or NULL */
  uint32_t n_chunks;            /* entries of chunks: at least the side's n_chunks (HY_ERR_INVALID_ARGUMENT
                                   otherwise - a filter built for a table that has grown since) */
  hy_row_id* out_row_ids;       /* device, capacity = side rows, or NULL: the TableScan's output as RowIDs
                                   {c, offset} (c = the side's chunk index) at the positions out_offsets would take -
                                   the PosLists of the scan's output chunks, written by the pass that ranks the matches
                                   (no expansion afterwards). Needs out_offsets and out_chunk_begin (scratch for
                                   passes that produce offsets first); out_offsets' contents are then unspecified.
                                   hy_scan_join_hash / prepared plans only (the exchange entry points refuse it) */
} hy_join_filter;

hy_status hy_scan_join_hash_workspace_size(const hy_join_side* build, const hy_join_filter* build_filter,
                                           const hy_join_side* probe, const hy_join_filter* probe_filter,
                                           const hy_join_params* params, size_t* bytes);
hy_status hy_scan_join_hash(const hy_join_side* build, const hy_join_filter* build_filter, const hy_join_side* probe,
                            const hy_join_filter* probe_filter, const hy_join_params* params, hy_row_id* out_build,
                            hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                            uint32_t* partition_counts, hy_join_result* result, void* workspace,
                            size_t workspace_bytes, hy_stream_t stream);

/*
 * Prepared plans: the same TableScan -> JoinHash over the same HBM-resident tables executed repeatedly (a prepared
 * statement). create() validates and plans both sides once and allocates the plan's own workspace; execute() runs the
 * whole pipeline - every kernel of hy_scan_join_hash - and stages the chunk / predicate descriptors to HBM only on its
 * first call (9,155 + 2,289 chunk descriptors at SF100: ~1.5 MB of host copies and DMA per call otherwise). The
 * descriptors' device pointers (column data, scan outputs) must stay valid while the plan lives. Results are exactly
 * hy_scan_join_hash's.
 */
typedef struct hy_join_plan_s* hy_join_plan_t;
hy_status hy_scan_join_plan_create(const hy_join_side* build, const hy_join_filter* build_filter,
                                   const hy_join_side* probe, const hy_join_filter* probe_filter,
                                   const hy_join_params* params, hy_join_plan_t* plan);
hy_status hy_scan_join_plan_execute(hy_join_plan_t plan, hy_row_id* out_build, hy_row_id* out_probe,
                                    uint64_t out_capacity, uint64_t* partition_begin, uint32_t* partition_counts,
                                    hy_join_result* result, hy_stream_t stream);
/* Points the plan's fused scans at new output buffers (out_offsets / out_chunk_begin / out_row_ids of the filters) for
 * the following executions - an operator re-executing a cached plan writes each execution's TableScan output into
 * buffers of its own. The filters' predicate chunks must equal the plan's (HY_ERR_INVALID_ARGUMENT otherwise), and
 * out_offsets / out_chunk_begin stay set or unset as at create; a rebound plan executes its launches eagerly from then
 * on (no hipGraph capture: a captured graph would hold the old pointers). Either filter NULL where the plan has none. */
hy_status hy_scan_join_plan_rebind(hy_join_plan_t plan, const hy_join_filter* build_filter,
                                   const hy_join_filter* probe_filter);
hy_status hy_scan_join_plan_destroy(hy_join_plan_t plan);

/* ---------------------------------------------------------------------------------------------------------------
 * Distributed JoinHash (one process per GPU; an RCCL all-to-all of records between the two steps)
 *
 * The radix partition id of a row (murmur2(key, seed) & (2^radix_bits - 1), radix_bits from the GLOBAL build size) is
 * split into digits from the most significant; the first digit has B = 2^w0 >= n_ranks buckets and rank r owns buckets
 * [r * B / n_ranks, (r + 1) * B / n_ranks) - hence a contiguous range of partitions, and the ranks' outputs
 * concatenated in rank order are the reference's output (join_hash.cpp:829-855: one chunk per partition, ascending).
 *
 * Step 1, every rank, each side: hy_join_exchange_partition writes the rank's rows of the side as 16-byte exchange
 * records {key (hashed type, 8-byte aligned), RowID} grouped by first-digit bucket (stable: row order inside a bucket)
 * and bucket_counts[b] (host, B entries). The RowID is the row's own (chunk_id of its hy_join_chunk, offset) or, for
 * a fused reference side, the referenced RowID from its PosList. The records for rank r are one contiguous range.
 * Step 2, every rank, after all-to-all (received buffer = the senders' ranges in sender order; counts[s * n_buckets +
 * j] = rows of local bucket j from sender s): hy_join_exchange_join partitions the received records further (stable,
 * bucket-major then sender then row order) and runs the LDS build/probe of the rank's n_buckets << (radix_bits - w0)
 * partitions. partition_begin / partition_counts as for hy_join_hash, indexed by local partition.
 * ------------------------------------------------------------------------------------------------------------- */
#define HY_EXCHANGE_RECORD_BYTES 16
hy_status hy_join_exchange_partition_workspace_size(const hy_join_side* side, const hy_join_params* params,
                                                    uint32_t n_ranks, size_t* bytes);
hy_status hy_join_exchange_partition(const hy_join_side* side, const hy_join_params* params, int32_t keep_nulls,
                                     uint32_t n_ranks, void* out_records, uint64_t* bucket_counts, void* workspace,
                                     size_t workspace_bytes, hy_stream_t stream);
hy_status hy_join_exchange_join_workspace_size(const uint64_t* build_counts, const uint64_t* probe_counts,
                                               uint32_t n_senders, uint32_t n_buckets, const hy_join_params* params,
                                               size_t* bytes);
hy_status hy_join_exchange_join(const void* build_records, const uint64_t* build_counts, const void* probe_records,
                                const uint64_t* probe_counts, uint32_t n_senders, uint32_t first_bucket,
                                uint32_t n_buckets, const hy_join_params* params, hy_row_id* out_build,
                                hy_row_id* out_probe, uint64_t out_capacity, uint64_t* partition_begin,
                                uint32_t* partition_counts, hy_join_result* result, void* workspace,
                                size_t workspace_bytes, hy_stream_t stream);
/* First-digit width of the distributed join's radix plan (buckets = 2^width). */
uint32_t hy_join_exchange_bucket_bits(uint32_t radix_bits, uint32_t n_ranks);

/*
 * Row-index exchange records (the default for data-table sides): {key (hashed type), uint32 global row index}, 8 bytes
 * for 4-byte hashed types (16 for 8-byte ones, alignment) - half the xGMI bytes of the RowID records above. The global
 * row index is row_base + the row's index in the side (chunks in order); every rank passes the index of its shard's
 * first row in the global table, so indexes are unique across ranks (< 2^32, < 2^31 with a fused scan).
 * hy_scan_join_exchange_partition is step 1 for a data-table side with an optional fused TableScan (filter as for
 * hy_scan_join_hash; its out_offsets / out_chunk_begin receive the scan output of this shard).
 * hy_join_exchange_join_rows is step 2; the global tables' chunk layouts (chunk sizes in global chunk-id order) turn
 * the received row indexes into the output RowIDs {global chunk id, offset}.
 * A reference side (an earlier operator's output: one PosList per chunk) takes part with fuse_dereference set: its
 * records carry the REFERENCED table's row (row_base + the row's index in side->referenced, chunks in order), as
 * write_output_columns dereferences a reference input (join_hash.cpp:584-592); no fused scan on such a side.
 */
uint32_t hy_join_exchange_row_record_bytes(int32_t hashed_type);
hy_status hy_scan_join_exchange_partition_workspace_size(const hy_join_side* side, const hy_join_filter* filter,
                                                         const hy_join_params* params, uint32_t n_ranks,
                                                         size_t* bytes);
hy_status hy_scan_join_exchange_partition(const hy_join_side* side, const hy_join_filter* filter,
                                          const hy_join_params* params, int32_t keep_nulls, uint32_t n_ranks,
                                          uint64_t row_base, void* out_records, uint64_t* bucket_counts,
                                          void* workspace, size_t workspace_bytes, hy_stream_t stream);
hy_status hy_join_exchange_join_rows_workspace_size(const uint64_t* build_counts, const uint64_t* probe_counts,
                                                    uint32_t n_senders, uint32_t n_buckets,
                                                    const hy_join_params* params, const uint32_t* build_chunk_sizes,
                                                    uint32_t n_build_chunks, const uint32_t* probe_chunk_sizes,
                                                    uint32_t n_probe_chunks, size_t* bytes);
hy_status hy_join_exchange_join_rows(const void* build_records, const uint64_t* build_counts,
                                     const void* probe_records, const uint64_t* probe_counts, uint32_t n_senders,
                                     uint32_t first_bucket, uint32_t n_buckets, const hy_join_params* params,
                                     const uint32_t* build_chunk_sizes, uint32_t n_build_chunks,
                                     const uint32_t* probe_chunk_sizes, uint32_t n_probe_chunks,
                                     hy_row_id* out_build, hy_row_id* out_probe, uint64_t out_capacity,
                                     uint64_t* partition_begin, uint32_t* partition_counts, hy_join_result* result,
                                     void* workspace, size_t workspace_bytes, hy_stream_t stream);

/*
 * Columns carried with the exchange (late materialisation across ranks). A distributed plan above a JoinHash needs
 * column values of rows that live on other ranks (TPC-H 3's projection reads o_orderdate / o_shippriority of the
 * build rows and l_extendedprice / l_discount of the probe rows, tpch_queries.cpp:101-106). The sender evaluates
 * them for its own records and ships them beside the records, in record order, with the same split sizes; the
 * receiver addresses them by the record's position in its receive buffer:
 *   hy_exchange_record_row_ids   sender: RowIDs {chunk, offset} of the records' payload rows (payload - row_base in
 *                                a table whose chunks have chunk_sizes) in record order - a PosList for hy_projection,
 *                                which then evaluates any column / expression of the shard in record order.
 *   hy_exchange_records_localize receiver: payload[i] := i (the record's position), after saving the old payloads to
 *                                old_payloads and the keys (hashed type, 4 or 8 bytes) to keys (each may be NULL).
 *                                hy_join_exchange_join_rows over the localized records with a layout of uniform chunks
 *                                over the receive buffer then emits RowIDs {position / chunk, position % chunk} into
 *                                the "received table", whose columns are the received attribute arrays.
 * record_bytes: hy_join_exchange_row_record_bytes(hashed type) (payload at byte offset record_bytes / 2).
 */
hy_status hy_exchange_record_row_ids(const void* records, uint64_t n, uint32_t record_bytes, uint64_t row_base,
                                     const uint32_t* chunk_sizes, uint32_t n_chunks, hy_row_id* out_row_ids,
                                     hy_stream_t stream);
hy_status hy_exchange_records_localize(void* records, uint64_t n, uint32_t record_bytes, void* keys,
                                       uint32_t* old_payloads, hy_stream_t stream);

/*
 * The exchange step between step 1 and step 2 over RCCL (xGMI), so that a C++ process runs the distributed join
 * without another runtime. One communicator per process (one process per GPU): rank 0 calls hy_comm_get_unique_id
 * and hands the 128 bytes to the other ranks over the host's own channel (the reference's network layer or a TCP
 * store), then every rank calls hy_comm_init on its device. Per side:
 *   hy_join_exchange_counts   all-gather of the B bucket counts (host in, host out: all_counts[s * B + b], N * B
 *                             entries; synchronises the stream);
 *   hy_join_exchange_records  sends this rank's records (grouped by bucket, as step 1 wrote them) to the buckets'
 *                             owners and receives, sender after sender, the records of its own buckets into
 *                             recv_records (device, recv_capacity records of record_bytes each); recv_counts (host,
 *                             N * n_local_buckets) is exactly the counts matrix step 2 takes; *recv_rows = rows
 *                             received. The abort decision is collective (one all-reduce of every rank's verdict
 *                             before any send): if ANY rank's buffer is too small every rank returns HY_ERR_CAPACITY
 *                             (each with its own *recv_rows set) and nothing is sent, so no rank is left blocked.
 * Asynchronous on `stream` like the other entry points; RCCL's send/recv round is stream-ordered.
 */
#define HY_COMM_ID_BYTES 128
typedef struct hy_comm_id {
  char bytes[HY_COMM_ID_BYTES];
} hy_comm_id;
typedef struct hy_comm_s* hy_comm_t;
hy_status hy_comm_get_unique_id(hy_comm_id* id);
hy_status hy_comm_init(hy_comm_t* comm, int32_t n_ranks, const hy_comm_id* id, int32_t rank);
hy_status hy_comm_destroy(hy_comm_t comm);
hy_status hy_join_exchange_counts(hy_comm_t comm, const uint64_t* bucket_counts, uint32_t n_buckets,
                                  uint64_t* all_counts, hy_stream_t stream);
hy_status hy_join_exchange_records(hy_comm_t comm, const void* records, uint32_t record_bytes,
                                   const uint64_t* all_counts, uint32_t n_buckets, void* recv_records,
                                   uint64_t recv_capacity, uint64_t* recv_counts, uint64_t* recv_rows,
                                   hy_stream_t stream);

/*
 * out[i] = rows[i] is NULL ? rows[i] : chunk_pos_lists[rows[i].chunk_id][rows[i].chunk_offset]
 * (reference write_output_columns, join_hash.cpp:584-592). chunk_pos_lists: DEVICE array of device PosList pointers.
 */
hy_status hy_dereference_row_ids(const hy_row_id* rows, uint64_t n, const hy_row_id* const* chunk_pos_lists,
                                 hy_row_id* out, hy_stream_t stream);


/* ---------------------------------------------------------------------------------------------------------------
 * Aggregate (GROUP BY + MIN / MAX / SUM / AVG / COUNT / COUNT(*) / COUNT(DISTINCT))
 *
 * Replaces Aggregate::_aggregate's group-id phase and the per-chunk aggregate loops (reference
 * src/lib/operators/aggregate.cpp:291-498, AggregateFunctionBuilder :133-249, traits
 * operators/aggregate/aggregate_traits.hpp:15-74) for all chunks of the input in one pass. The output is one
 * record of 64-bit words per group; the caller (the Aggregate operator) orders the groups the way the reference's
 * std::unordered_map iterates them (from the first-row words) and writes the output columns
 * (write_aggregate_values / _write_groupby_output, aggregate.cpp:622-820).
 *
 * Record layout (hy_aggregate_layout reports the word offsets):
 *   [0, n_groupby)  key words: group-by value bits (4-byte types zero-extended, -0.0 folded into 0.0), 0 if NULL
 *   n_groupby + 0   NULL mask of the group-by values (bit j = group-by j is NULL)
 *   n_groupby + 1   first row: smallest input row index of the group (input rows are numbered chunk by chunk)
 *   n_groupby + 2   last row: largest input row index of the group
 *   n_groupby + 3   rows of the group (= COUNT(*))
 *   per aggregate a at word agg_word[a]:
 *     COUNT, COUNT(DISTINCT): count
 *     MIN, MAX:               non-NULL count, order-preserving bits of the extreme value (hy_agg_decode_ordered)
 *     SUM, AVG of integers:   non-NULL count, int64 sum (two's complement)
 *     SUM, AVG of floats:     non-NULL count, non-finite flags (1 +inf, 2 -inf, 4 NaN), then agg_limbs[a] signed
 *                             64-bit limbs; limb i has weight 2^(32 i + agg_emin[a]). hy_agg_float_sum rounds the
 *                             exact sum once to double. One more word follows the limbs (device scratch for
 *                             integer-valued rows, always 0 in returned records).
 *     COUNT(*):               no words (use the rows word)
 * In dense mode (every group-by column arrives as integer codes with a domain, product of (domain + 1) <= 64) the
 * key words of a group are its codes.
 * ------------------------------------------------------------------------------------------------------------- */
/* Expression nodes (postfix programs) of hy_projection and of expression columns of hy_aggregate; see the Projection
 * section below for their semantics. */
enum { HY_EXPR_COLUMN = 0, HY_EXPR_VALUE = 1, HY_EXPR_ADD = 2, HY_EXPR_SUB = 3, HY_EXPR_MUL = 4, HY_EXPR_DIV = 5,
       HY_EXPR_MOD = 6 };
enum { HY_EXPR_MAX_NODES = 32, HY_EXPR_MAX_DEPTH = 8 };

typedef struct hy_expr_node {
  int32_t kind;       /* HY_EXPR_* */
  int32_t type;       /* HY_TYPE_* of the node's value (0: NULL literal) */
  int32_t calc_type;  /* arithmetic: HY_TYPE_* the operation is computed in */
  int32_t column;     /* COLUMN: index into hy_agg_input.columns */
  uint64_t value;     /* VALUE: the literal's bits in `type` (int32/float in the low 4 bytes) */
} hy_expr_node;

enum { HY_AGG_MIN = 0, HY_AGG_MAX = 1, HY_AGG_SUM = 2, HY_AGG_AVG = 3, HY_AGG_COUNT = 4, HY_AGG_COUNT_DISTINCT = 5 };
enum { HY_AGG_MAX_COLUMNS = 16, HY_AGG_MAX_GROUPBY = 8, HY_AGG_MAX_AGGREGATES = 16, HY_AGG_MAX_POS_GROUPS = 8 };

typedef struct hy_agg_column {
  int32_t value_type;                /* HY_TYPE_* of the values (string columns arrive as HY_TYPE_INT32 codes) */
  int32_t pos_group;                 /* -1: data input (chunks[c] is input chunk c); else the PosList group through
                                        which this column's values are referenced (chunks[] = referenced chunks) */
  const hy_column_chunk* chunks;     /* HOST array of n_chunks device column chunks */
  uint32_t n_chunks;
  uint32_t domain;                   /* group-by only: 0, or every non-NULL value is an integer code < domain */
  /* Expression column (n_nodes > 0): each row's value is the postfix program over the input's other, plain columns
   * (hy_expr_node semantics of hy_projection: the reference's Projection feeding the Aggregate, evaluated inside the
   * aggregation instead of materialised); value_type = the program's result type; chunks / pos_group unused. */
  const hy_expr_node* program;       /* HOST array of n_nodes nodes, or NULL */
  uint32_t n_nodes;
  uint32_t reserved;
} hy_agg_column;

typedef struct hy_agg_input {
  uint32_t n_chunks;                 /* input chunks */
  const uint32_t* chunk_sizes;       /* HOST: rows per input chunk (PosList length for reference input) */
  const hy_row_id* const* pos_lists; /* HOST: n_pos_groups * n_chunks device PosLists, [g * n_chunks + c] */
  uint32_t n_pos_groups;
  const hy_agg_column* columns;      /* HOST */
  uint32_t n_columns;
  /* Fused TableScan (the plan TableScan -> [Projection ->] Aggregate as one pass, reference table_scan.cpp:78-164
   * feeding aggregate.cpp:291-498): NULL, or - for a data input (n_pos_groups == 0) on the dense expression path -
   * one predicate chunk per input chunk (hy_scan_chunk as for hy_table_scan: op + search_vid of the host's dictionary
   * rewrite, or a value compare with *filter_constant of filter_value_type). Rows that do not match take no part,
   * exactly as if the Aggregate read the scan's output; the first / last row words number the input's rows (an
   * order-preserving renumbering of the scan output's). Other paths return HY_ERR_UNSUPPORTED. */
  const hy_scan_chunk* filter;       /* HOST, n_chunks entries */
  int32_t filter_value_type;
  const void* filter_constant;       /* HOST */
} hy_agg_input;

typedef struct hy_agg_def {
  int32_t function;                  /* HY_AGG_* */
  int32_t column;                    /* index into hy_agg_input.columns; -1 for COUNT(*) */
} hy_agg_def;

typedef struct hy_agg_params {
  const int32_t* groupby;            /* HOST: indexes into hy_agg_input.columns */
  uint32_t n_groupby;
  const hy_agg_def* aggregates;      /* HOST */
  uint32_t n_aggregates;
  uint64_t group_bound;              /* expected number of groups (sizes the hash table); 0 = derived: the product
                                        of the group-by columns' dictionary sizes when every group-by column is
                                        dictionary-encoded, else min(rows, the groups 2 GiB of records hold,
                                        at least 2^20). Exceeding it returns
                                        HY_ERR_GROUP_BOUND with a larger bound; the call has no other effect. */
} hy_agg_params;

typedef struct hy_agg_layout {
  uint32_t words;                            /* 64-bit words per group record */
  uint32_t dense;                            /* 1 if the dense (code-indexed) path is used */
  uint32_t agg_word[HY_AGG_MAX_AGGREGATES];
  int32_t agg_emin[HY_AGG_MAX_AGGREGATES];
  uint32_t agg_limbs[HY_AGG_MAX_AGGREGATES];
} hy_agg_layout;

hy_status hy_aggregate_layout(const hy_agg_input* input, const hy_agg_params* params, hy_agg_layout* layout);
hy_status hy_aggregate_workspace_size(const hy_agg_input* input, const hy_agg_params* params, size_t* bytes);
/*
 * out_records: device, out_capacity * layout.words words. *n_groups (host) receives the number of groups; the call
 * synchronizes the stream. HY_ERR_CAPACITY if more than out_capacity groups (*n_groups holds the number needed).
 */
hy_status hy_aggregate(const hy_agg_input* input, const hy_agg_params* params, uint64_t* out_records,
                       uint64_t out_capacity, uint64_t* n_groups, void* workspace, size_t workspace_bytes,
                       hy_stream_t stream);
/* ---------------------------------------------------------------------------------------------------------------
 * Projection of arithmetic expressions (reference src/lib/operators/projection.cpp:39-87 evaluating
 * ArithmeticExpression / PQPColumnExpression / ValueExpression through ExpressionEvaluator,
 * expression/evaluation/expression_evaluator.cpp:105-120, :795-830, expression_functors.hpp:104-180).
 *
 * The expression is a postfix program over the columns of a hy_agg_input (data chunks or columns referenced through
 * PosList groups, exactly as for hy_aggregate). Every node carries the reference's types:
 *   type       the node's result type: a column's / literal's type; for arithmetic expression_common_type(l, r)
 *              (expression/expression_utils.cpp:116-136)
 *   calc_type  arithmetic only: the type the operation runs in, std::common_type of the operands' types (the
 *              functors compute Functor<std::common_type_t<A, B>>(a, b) and assign it to the result type)
 * NULL logic: + - * are NULL if an operand is NULL; / and % also when the divisor is 0 (integral % or fmod).
 * A NULL literal is a VALUE node with type 0 (every row NULL).
 * Output: values[r] (result type) and nulls[r] (1 = NULL; may be NULL when the expression is not nullable) for input
 * row r, rows numbered chunk by chunk. Values of NULL rows are unspecified.
 * ------------------------------------------------------------------------------------------------------------- */
hy_status hy_projection_workspace_size(const hy_agg_input* input, size_t* bytes);
hy_status hy_projection(const hy_agg_input* input, const hy_expr_node* program, uint32_t n_nodes, void* out_values,
                        uint8_t* out_nulls, void* workspace, size_t workspace_bytes, hy_stream_t stream);
/* Several expressions over the same input in one launch, as the reference's Projection evaluates every expression of
 * its node per chunk (projection.cpp:52-85): program i (n_nodes[i] nodes) writes out_values[i] / out_nulls[i]
 * (out_nulls may be NULL, or hold NULL entries). The rows' chunks, RowIDs and column reads are shared by the programs;
 * each result equals hy_projection's for that program. n_programs <= HY_PROJ_MAX_OUTPUTS; the workspace is
 * hy_projection_workspace_size's. */
enum { HY_PROJ_MAX_OUTPUTS = 16 };
hy_status hy_projection_multi(const hy_agg_input* input, const hy_expr_node* const* programs, const uint32_t* n_nodes,
                              uint32_t n_programs, void* const* out_values, uint8_t* const* out_nulls, void* workspace,
                              size_t workspace_bytes, hy_stream_t stream);

/* Host helpers: the correctly rounded double of an exact limb sum, and the value bits behind an ordered word. */
/*
 * Multi-GPU Aggregate: merges the group records of n_parts partial aggregates (same params / layout; parts[p]: HOST
 * records of part p, part_groups[p] of them; part_row_base[p]: added to the first / last row words, the part's first
 * row in the global row numbering; may be NULL) into out (HOST, out_capacity records). Exact: counts and integer sums
 * add, float-sum limbs add and are carry-normalised (hy_agg_float_sum of a merged record = that of one aggregate over
 * all rows), MIN / MAX combine the parts that have values. COUNT(DISTINCT) -> HY_ERR_UNSUPPORTED. Groups appear in
 * order of first appearance over the parts; *n_out = merged groups (HY_ERR_CAPACITY if more than out_capacity).
 */
hy_status hy_aggregate_merge(const hy_agg_params* params, const hy_agg_layout* layout, const uint64_t* const* parts,
                             const uint64_t* part_groups, const uint64_t* part_row_base, uint32_t n_parts,
                             uint64_t* out, uint64_t out_capacity, uint64_t* n_out);
hy_status hy_agg_float_sum(const uint64_t* limbs, uint32_t n_limbs, int32_t emin, uint64_t special, double* out);
/* hy_agg_float_sum over n_records HOST group records of `words` words each: out[g] = the float SUM of the aggregate
 * whose words start at sum_word of record g (its non-finite flags at sum_word + 1, n_limbs limbs from sum_word + 2).
 * The host side of reading a large GROUP BY result back (TPC-H 3's 1.1 M groups at SF100). */
hy_status hy_agg_float_sums(const uint64_t* records, uint64_t n_records, uint32_t words, uint32_t sum_word,
                            uint32_t n_limbs, int32_t emin, double* out);
uint64_t hy_agg_decode_ordered(uint64_t ordered, int32_t value_type);

#ifdef __cplusplus
}
#endif

#endif /* HYRISE_AMD_H_ */
