/* tfrg_status.h — per-record status codes shared by the device path (libtfrg), the host
 * mirror (tfr_reader) and the test oracle (oracle/tfrg_oracle.c).
 *
 * Codes 1..14 mirror, one for one, the exceptions the reference raises on the decode path
 * (Python message text in tfr_reader/_status.py):
 *   src/tfr_reader/cython/decoder.pyx:49   'Too many bytes when decoding varint.'
 *   decoder.pyx:79   'Unexpected end of buffer when reading fixed64.'
 *   decoder.pyx:89   'Unexpected end of buffer when reading length-delimited field.'
 *   decoder.pyx:98   'Unexpected end of buffer when reading fixed32.'
 *   decoder.pyx:104  'Unsupported wire type: {}'            (aux = the wire type)
 *   decoder.pyx:123  'Unexpected wire type for field features'
 *   decoder.pyx:147  'Unexpected wire type for field feature'
 *   decoder.pyx:199  'Unexpected field number in Feature'
 *   decoder.pyx:220  'Unexpected wire type in BytesList'
 *   decoder.pyx:264  'Unexpected wire type in FloatList'
 *   decoder.pyx:297  'Unexpected wire type in Int64List'
 *   decoder.pyx:164  UnicodeDecodeError from bytes(key).decode('utf-8')  (aux = key off<<32 | len)
 *   example/feature.py:106  AttributeError: Example(features=None)  (no Features field)
 *   reader.py:48-49  OSError: empty read for the byte range
 * Code 15 exists only under TFRG_FLAG_STRICT_CRC (a TFRecord-spec integrity check the reference
 * does not have). tfrg_status_message / tfrg_status_exception (tfrg.h) give the text.
 * Codes 32..35 are shapes on which the reference has undefined behaviour (segfault, reads past
 * the bytes object, non-terminating parse). The build reports them instead.
 */
#ifndef TFRG_STATUS_H
#define TFRG_STATUS_H

enum tfrg_status {
  TFRG_OK = 0,
  TFRG_ERR_VARINT_TOO_MANY = 1,
  TFRG_ERR_EOB_FIXED64 = 2,
  TFRG_ERR_EOB_LEN = 3,
  TFRG_ERR_EOB_FIXED32 = 4,
  TFRG_ERR_WIRE_TYPE = 5,
  TFRG_ERR_WT_FEATURES = 6,
  TFRG_ERR_WT_FEATURE = 7,
  TFRG_ERR_FEATURE_FIELD = 8,
  TFRG_ERR_WT_BYTES_LIST = 9,
  TFRG_ERR_WT_FLOAT_LIST = 10,
  TFRG_ERR_WT_INT64_LIST = 11,
  TFRG_ERR_KEY_UTF8 = 12,
  TFRG_ERR_FEATURES_NONE = 13,
  TFRG_ERR_READ = 14,
  TFRG_ERR_CRC = 15,            /* TFRG_FLAG_STRICT_CRC: length field / masked CRC-32C mismatch
                                   (not a reference error: the reference never checks CRCs;
                                   aux = the record's verdict bits)                            */
  /* reference undefined behaviour */
  TFRG_UB_EMPTY_FEATURE = 32,   /* decoder.pyx:177 fields[0] of an empty vector (segfault)   */
  TFRG_UB_SHORT_MAP_ENTRY = 33, /* decoder.pyx:163,165 fields[0]/[1] out of range (segfault) */
  TFRG_UB_NEGATIVE_LENGTH = 34, /* decoder.pyx:85-92 negative varint length moves pos back   */
  TFRG_UB_READ_PAST_END = 35,   /* decode_varint (decoder.pyx:34-50) past the NUL terminator */
  /* build-internal (never surfaced as a decode result) */
  TFRG_ST_SCHEMA_MISS = 64,     /* a key/kind not in the device key table: intern and re-run  */
  TFRG_ST_LIMIT = 65,           /* a build limit (e.g. > 65534 keys in one record)            */
  TFRG_ST_INTERNAL = 66         /* a device-internal list location outside its record (a stale or
                                   corrupt count / loc word): the list is not walked; aux = slot */
};

/* Feature kinds, numbered as the tf.train.Feature oneof field numbers (decoder.pyx:179-197). */
enum tfrg_kind { TFRG_KIND_NONE = 0, TFRG_KIND_BYTES = 1, TFRG_KIND_FLOAT = 2, TFRG_KIND_INT64 = 3 };

/* Framing verdict bits (per record). CRC-32C is absent from the reference. */
enum tfrg_verdict {
  TFRG_V_LEN_MATCH = 1u,  /* u64 length field == end - start - 16                 */
  TFRG_V_LEN_CRC = 2u,    /* masked CRC-32C of the 8 length bytes matches          */
  TFRG_V_DATA_CRC = 4u,   /* masked CRC-32C of the payload matches                 */
  TFRG_V_TRUNCATED = 8u   /* range ran past the end of the buffer (clamped)        */
};

/* tfrg_info.implicit_cols (tfrg.h): columns an optimistic decode did not store */
#define TFRG_IMPLICIT_STATUS 1u /* status 0, aux 0, verdict LEN_MATCH | LEN_CRC | DATA_CRC for every record */
#define TFRG_IMPLICIT_ORDER 2u  /* every slot's order word the same for every record */
#define TFRG_IMPLICIT_BYTES_LEN 4u /* every bytes_list slot one element of one length for every record */

#endif
