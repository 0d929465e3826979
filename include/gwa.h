/* gwa.h -- C ABI of the MI355X-native genome-weaver `align` path (drop-in boundary).
 *
 * Replaces, for the single-end FM-index path, the reference's Java plugin surface:
 *   interface Aligner { void align(Read read, Reporter out) }      A/Aligner.java:30-33
 *   Align.query(...) strategy selection (-m bsf, -m sf)              A/Align.java:112-140
 *   Reporter.emit -> SAMOutput.emit -> AlignmentRecord.toSAMLine     J/parallel/Reporter.java:27-30,
 *                                                                    A/SAMOutput.java:73-82
 *   FMIndexOnGenome.load / buildFromSequence                         A/FMIndexOnGenome.java:60-115
 *   SequenceBoundary.toSAMHeader                                     A/SequenceBoundary.java:81-87
 * (paths relative to align/src/main/java/org/utgenome/weaver/; A = align/, J = .)
 *
 * Conventions: 0 = OK, negative = error (message via gwa_last_error, thread-local).  A read on
 * which the reference would throw fails the whole batch (the reference aborts the run,
 * S/BidirectionalSuffixFilter.java:264-267).  Results are in input order.  Calls on one index
 * handle are serialised (one HIP stream per handle, one handle per GPU).  Plain pointers and
 * sizes only; no C++ or torch types cross this boundary.
 */
#ifndef GWA_H
#define GWA_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gwa_index gwa_index_t;
typedef struct gwa_batch gwa_batch_t;

/* AlignmentConfig + AlignmentScoreConfig (A/AlignmentConfig.java:40-72, A/AlignmentScoreConfig.java:37-77);
 * defaults from gwa_config_default: k 0.1, bsf, besthit, L 5, g 1, e 4, s 1, M 1, N 3, G 11, E 4, S 11, P 5, W 31 */
typedef struct {
  float k;
  int32_t strategy;    /* 0 = bsf (-m bsf), 1 = sf (-m sf, S/SuffixFilter.java); others are rejected */
  int32_t report_type; /* 0 besthit, 1 allhits, 2 topL (-R) */
  int32_t top_l;       /* -L */
  int32_t num_gap_open, num_gap_ext, num_split; /* -g -e -s */
  int32_t match, mismatch, gap_open, gap_ext, split_open; /* -M -N -G -E -S */
  int32_t indel_end_skip, band_width; /* -P -W */
} gwa_config_t;

/* A batch of reads, SoA, caller-owned.  Read i = name[name_off[i], name_off[i+1]), etc.
 * qual may be NULL: no read has a quality (SAM QUAL "*", as for FASTA input / -q queries).
 * qual_null (optional, may be NULL) marks single reads without one, one byte per read: nonzero =
 * read i's Read.getQual(0) is null (R/SingleEndRead.java:74-76, FASTA records) and its QUAL prints
 * "*" (R/AlignmentRecord.java:157) -- its qual_off range is ignored.  Zero-initialise the struct. */
typedef struct {
  uint32_t n;
  const char *name, *seq, *qual;
  const uint64_t *name_off, *seq_off, *qual_off;
  const uint8_t *qual_null;
} gwa_reads_t;

/* Reads parsed by the library from FASTA / FASTQ text (gwa_reads_parse); `reads` points into
 * library-owned blobs until gwa_reads_free.  Replaces the reference's read-file readers
 * (R/ReadReaderFactory.java:126-151, utgb FastqReader: unvendored, record rules in reads_io.cpp). */
typedef struct {
  gwa_reads_t reads;
  void *priv;
} gwa_read_buf_t;

/* One SAM record as the fields of the reference's AlignmentRecord (R/AlignmentRecord.java:44-79:
 * readName, chr, strand, start, end, numMismatches, cigar, querySeq, qual, score = 1, numBestHits,
 * alignmentState, split), so a JVM binding can build the objects SAMOutput.emit prints
 * (A/SAMOutput.java:73-82).  String fields are (offset, length) into gwa_results_t.sam. */
typedef struct {
  uint32_t read;          /* input index of the read */
  uint32_t flag;          /* SAM FLAG */
  int32_t ref;            /* contig index of chr; -1 = "*" */
  int32_t pos;            /* start */
  int32_t end;            /* end where the text fixes it (a split record: POS + TLEN of its first line), else pos */
  int32_t strand;         /* 0 = Strand.FORWARD, 1 = REVERSE (FLAG 0x10) */
  int32_t nm;             /* numMismatches: NM:i, -1 when the line has none */
  int32_t x0;             /* numBestHits: X0:i, 0 when absent (unmapped) */
  int32_t split;          /* index (in the record array) of this record's split record, -1 = none */
  int32_t is_split;       /* 1: this record is another record's split (emit the first one only) */
  int32_t qual_null;      /* 1: QUAL is "*" (qual == null) */
  int32_t pad_;
  uint64_t line_off, name_off, cigar_off, seq_off, qual_off, state_off;
  uint32_t line_len, name_len, cigar_len, seq_len, qual_len, state_len;
} gwa_record_t;

/* Library-owned SAM text (no header), in input order; read i's lines are
 * sam[line_off[i], line_off[i+1]).  Free with gwa_results_free.  records / n_records are filled on
 * request by gwa_results_records (NULL / 0 until then).  paired = 1: results of a paired-end batch,
 * unit i = pair i, two mate lines (mate 1, mate 2), never split records. */
typedef struct {
  uint32_t n_reads;
  char *sam;
  uint64_t sam_len;
  uint64_t *line_off; /* n_reads + 1 */
  gwa_record_t *records;
  uint64_t n_records;
  uint32_t paired;
} gwa_results_t;

/* Per-batch counters (instrumentation for SURVEY.md §8d roofline accounting). */
typedef struct {
  double kernel_ms;        /* device time of all kernels of gwa_batch_run: encode + align (HIP events) */
  double quickscan_ms;     /* fm_quickscan kernel */
  double search_ms;        /* bsf_search kernels (all tiers) */
  uint64_t fm_searches;    /* numFMIndexSearches summed over reads */
  uint64_t quick_steps;    /* FMQuickScan steps */
  uint64_t blocks;         /* 64-B Occ blocks read (algorithmic bytes = 64 * blocks) */
  uint64_t quick_blocks;   /* of which by fm_quickscan */
  uint64_t states;         /* search states created */
  uint64_t sa_reads;       /* 4-B suffix-array gathers (exact hits + verifications) */
  uint32_t tier_reads[4];  /* reads processed per capacity tier */
  uint32_t n_mapped, n_unmapped;
  uint64_t kmer_lookups;   /* 8-B k-mer interval-table reads by fm_quickscan */
  uint64_t quick_short_steps; /* FMQuickScan steps answered without Occ blocks (k-mer table, single-row text compare) */
  uint64_t quick_sa_reads; /* of sa_reads, by fm_quickscan */
  uint64_t search_short_steps; /* search FM steps answered by one text character (single-row states) */
  float tier_ms[4];        /* search time per capacity tier (HIP events) */
  uint64_t num_sw;         /* DP verifications (alignBlockDetailed calls) */
  uint64_t verify_bytes;   /* SURVEY.md 8(d) bytes of those verifications (reference window + Peq) */
  uint64_t quick_text_runs; /* fm_quickscan text-mode runs (one 32-base 2-bit text window + N flags each) */
  double encode_ms;        /* read encoding on the device at the start of gwa_batch_run (part of kernel_ms) */
  double format_ms;        /* the last SAM formatting of the batch on the device (gwa_batch_format / results) */
  double rescue_ms;        /* paired-end batches: pair choice + mate rescue kernels (part of kernel_ms) */
  uint64_t heavy_pairs;    /* paired-end batches: pairs chosen by the sorted sweep (> 64 candidate combinations) */
  uint64_t rescue_window_skipped; /* paired-end: mate rescues not tried, because the mate is longer than
                                   * 256 bp or the window the insert range allows (max_insert - min_insert
                                   * + m + 2 kr) exceeds 320 bases */
} gwa_batch_stats_t;

void gwa_config_default(gwa_config_t *cfg);
const char *gwa_last_error(void);
int gwa_device_count(void);

/* Build an index from FASTA text (the `bwt` command: PackFasta + cyclic SA + BWT) and place
 * it in HBM of `device`. */
int gwa_index_build_fasta(const char *fasta_text, uint64_t len, int device, gwa_index_t **out);
/* Same, from a file (the `-r` argument): a FASTA file, or an index saved by gwa_index_save (recognised
 * by its magic), which skips the FASTA parse. */
int gwa_index_open(const char *fasta_path, int device, gwa_index_t **out);
/* Save an index (2-bit text, N bitmap, contig table; the suffix arrays and Occ blocks are rebuilt on
 * the GPU at load).  Plays the role of the reference's `bwt` command output (A/BWTransform.java:72-179,
 * A/BWTFiles.java:40-80) in this build's own format. */
int gwa_index_save(const gwa_index_t *ix, const char *path);
/* Same, from codes 0..4 (A,C,G,T,N) and a contig table (names + lengths, concatenated in order). */
int gwa_index_build_codes(const uint8_t *codes, uint64_t n, int32_t n_contigs, const char *const *names,
                          const int64_t *lengths, int device, gwa_index_t **out);
uint64_t gwa_index_text_size(const gwa_index_t *ix);
uint64_t gwa_index_device_bytes(const gwa_index_t *ix);
/* Export the cyclic suffix array of strand 0 (text) or 1 (reversed text), n entries. */
int gwa_index_export_sa(const gwa_index_t *ix, int strand, uint32_t *out);
int gwa_sam_header(const gwa_index_t *ix, char **text, uint64_t *len);
void gwa_index_close(gwa_index_t *ix);

/* One call per batch: H2D, align on the GPU, D2H, SAM formatting. */
int gwa_align_batch(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *reads, gwa_results_t *out);
void gwa_results_free(gwa_results_t *r);
/* Fill r->records (one gwa_record_t per SAM line, in text order) from the SAM text of r. */
int gwa_results_records(const gwa_index_t *ix, gwa_results_t *r);
void gwa_free(void *p);

/* Parse the complete records of text[0, len): format 0 = FASTA, 1 = FASTQ.  With final = 0 the
 * last record may continue past len and is left for the next call; *consumed = bytes parsed
 * (the caller keeps text[*consumed, len) in front of its next chunk).  <0 on a malformed record. */
int gwa_reads_parse(const char *text, uint64_t len, int format, int final, gwa_read_buf_t *out, uint64_t *consumed);
void gwa_reads_free(gwa_read_buf_t *b);

/* Split form used by bench.py: upload once (reads resident in HBM), run the kernels (timed),
 * then fetch results. */
int gwa_batch_create(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *reads, gwa_batch_t **out);
int gwa_batch_run(gwa_batch_t *b);
/* Paired-end batch (config C5; the build's own design -- the reference has no paired-end path,
 * R/ReadReaderFactory.java:60-84): mate1[i] and mate2[i] form pair i.  Each mate is aligned as a
 * single-end read (-m bsf, every best hit kept); the pair of hits on one contig, opposite strands,
 * forward-reverse, with template length in [min_insert, max_insert] and the fewest differences wins
 * (rules: oracle/gwa_oracle.cpp orc_align_pairs).  Results hold two SAM lines per pair (n_reads =
 * pairs, line_off per pair) with mate fields and TLEN.
 * Mate rescue (rule 3) aligns the other mate inside the window the insert range allows next to the
 * anchor; it is tried for mates of at most 256 bp and windows of at most 320 bases (max_insert -
 * min_insert + m + 2 max(k, m / 10); the default 210-390 gives 300 for 100 bp mates).  Longer mates
 * and wider windows skip the rescue and are counted in gwa_batch_stats_t.rescue_window_skipped. */
int gwa_batch_create_pairs(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *mate1, const gwa_reads_t *mate2,
                           int32_t min_insert, int32_t max_insert, gwa_batch_t **out);
/* One call per paired batch: create_pairs + run + results. */
int gwa_align_pairs(gwa_index_t *ix, const gwa_config_t *cfg, const gwa_reads_t *mate1, const gwa_reads_t *mate2,
                    int32_t min_insert, int32_t max_insert, gwa_results_t *out);
int gwa_batch_stats(gwa_batch_t *b, gwa_batch_stats_t *st);
int gwa_batch_results(gwa_batch_t *b, gwa_results_t *out);
/* The batch's SAM text written in HBM only (paired-end: pairing included); *sam_bytes = its size.
 * For timing the device side of the reporting path; gwa_batch_results copies the text out. */
int gwa_batch_format(gwa_batch_t *b, uint64_t *sam_bytes);
/* Device-to-device copy of the batch's SAM text as the last gwa_batch_format wrote it in HBM (input
 * order, no header) into dst, device memory of the batch's GPU with room for *len bytes; with dst NULL
 * only *len is set.  Fails unless the last formatting of the batch was gwa_batch_format.  For a
 * device-side gather of the SAM of several GPUs over RCCL / xGMI (genome-weaver-align_amd/dist.py
 * gather_sam_device; SURVEY.md §8e's optional collective). */
int gwa_batch_sam_copy(gwa_batch_t *b, void *dst, uint64_t *len);
/* SAM for reads [first, first+count) only (n_reads = count). */
int gwa_batch_results_range(gwa_batch_t *b, uint32_t first, uint32_t count, gwa_results_t *out);
void gwa_batch_free(gwa_batch_t *b);
/* SAM for the reads idx[0..count) in that order (n_reads = count). */
int gwa_batch_results_select(gwa_batch_t *b, const uint32_t *idx, uint32_t count, gwa_results_t *out);
/* Instrumentation: per-read counters after gwa_batch_run, GWA_READ_COUNTERS int32 per read:
 * [0] status, [1] fm_searches (numFMIndexSearches), [2] quick_steps (FMQuickScan steps),
 * [3] quickscan Occ blocks, [4] search Occ blocks, [5] search states, [6] SA gathers, [7] hits,
 * [8..11] quick-scan mismatches / longest-match start (forward, reverse; searched reads only),
 * [12] deepest search tier (-1 = finished in the quick scan), [13] k-mer table lookups,
 * [14] quick-scan steps answered without Occ blocks, [15] search steps answered from the text,
 * [16] DP verifications (numSW), [17] SURVEY.md 8(d) verify bytes, [18..19] 0. */
#define GWA_READ_COUNTERS 20
int gwa_batch_read_counters(gwa_batch_t *b, int32_t *out);

/* ---- Multi-device driver and overlapped host pipeline (8(f) row 2) ----
 * Replaces the reference's single-threaded read loop (A/Align.java:174-196: ReadReaderFactory ->
 * PassReadToAligner -> Aligner.align -> SAMOutput.emit, one read at a time).  A pipeline holds n_ix
 * index handles -- one per GPU, each a full replica -- and deals read batches of batch_reads reads
 * to them as they become free (workers_per_device host threads per handle overlap one batch's set-up
 * and SAM formatting with another's kernels).  Output is in input order, byte-identical to a
 * single-handle run.  The handles must outlive the pipeline.  workers_per_device <= 0 means 3.
 * The first gwa_pipeline_align_file call pins the read-text buffers a file run keeps in flight (sized
 * from the file, at most a quarter of the host's available memory; about 5.4 GB for a large file on
 * one device); they and each worker's pinned SAM buffer are kept for later calls.  In-memory runs
 * (gwa_pipeline_align) pin nothing.  Output to an O_APPEND descriptor or a pipe is written in batch
 * order with write(); to a regular file, each batch at its offset with pwrite(). */
typedef struct gwa_pipeline gwa_pipeline_t;
typedef struct {
  uint64_t reads, batches;
  double wall_s;               /* the last align / align_file call */
  double read_s;               /* of which reading (and decompressing) the read file */
  double device_kernel_s[16];  /* per handle: time inside gwa_batch_run */
  /* align_file stage times, summed over worker threads: read parse, batch set-up (H2D + encode),
   * SAM formatting + D2H, output writes, and waiting for the batch-order output position */
  double parse_s, setup_s, format_s, write_s, order_wait_s;
  double frame_s;  /* reader thread: framing the text into batches of complete records */
  uint64_t pinned_bufs;  /* align_file: pinned read-text buffers large enough for this file's chunks */
} gwa_pipeline_stats_t;
int gwa_pipeline_open(gwa_index_t *const *ix, int n_ix, const gwa_config_t *cfg, uint32_t batch_reads,
                      int workers_per_device, gwa_pipeline_t **out);
/* SAM (no header) of any number of reads, in input order. */
int gwa_pipeline_align(gwa_pipeline_t *p, const gwa_reads_t *reads, gwa_results_t *out);
/* A FASTA / FASTQ file (.fa .fasta .fan .fastq .fq, optionally .gz or .snap; ReadReaderFactory.createReader,
 * R/ReadReaderFactory.java:126-151) streamed through the devices; SAM records (no header) are
 * written to fd in input order.  *n_reads = reads aligned. */
int gwa_pipeline_align_file(gwa_pipeline_t *p, const char *path, int fd, uint64_t *n_reads);
/* The same over the bytes [begin, end) of a plain (not .gz / .snap) read file, which must start at a record
 * (gwa_reads_shard_range gives such ranges). */
int gwa_pipeline_align_file_range(gwa_pipeline_t *p, const char *path, int fd, uint64_t begin, uint64_t end,
                                  uint64_t *n_reads);
/* One process per GPU (C3; the reference's one read loop, A/Align.java:174-196, split by reads): the
 * byte range [*begin, *end) of shard `shard` of `nshards` contiguous shards of a plain FASTQ / FASTA
 * file, cut at record starts, so that the shards' SAM files concatenated in shard order equal a
 * one-process run's (the header belongs to shard 0). */
int gwa_reads_shard_range(const char *path, uint32_t shard, uint32_t nshards, uint64_t *begin, uint64_t *end);
/* The bytes of a `.snap` file (R/ReadReaderFactory.java:130-139, org.xerial.snappy.SnappyInputStream):
 * a snappy-java stream (magic header, then length-prefixed Snappy blocks) or one bare Snappy block,
 * decompressed into *out (malloc'd, NUL-terminated; gwa_free).  Host only, no device needed. */
int gwa_snappy_decompress(const uint8_t *in, uint64_t n, char **out, uint64_t *out_len);
int gwa_pipeline_stats(const gwa_pipeline_t *p, gwa_pipeline_stats_t *st);
void gwa_pipeline_close(gwa_pipeline_t *p);

#ifdef __cplusplus
}
#endif
#endif /* GWA_H */
