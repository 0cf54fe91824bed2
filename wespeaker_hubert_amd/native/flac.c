/* FLAC decoder for the extraction front door (host code, CPU data pipeline).
 *
 * The reference decodes FLAC members of its shards / raw lists with
 * torchaudio.load (dataset/processor.py:96-110, AUDIO_FORMAT_SETS :34); this is
 * the host-side decoder behind wespeaker_hubert_amd.audio.load_audio for them.
 * It follows the published FLAC format specification (RFC 9639):
 *   - "fLaC" marker, metadata blocks (STREAMINFO read, the others skipped);
 *   - frames: sync 0b11111111111110, fixed or variable block size, block size /
 *     sample rate / channel assignment / sample size codes, UTF-8 coded frame or
 *     sample number, CRC-8 (poly 0x07) over the header;
 *   - subframes CONSTANT, VERBATIM, FIXED (order 0..4), LPC (order 1..32,
 *     precision, shift), wasted bits; residual coding methods 0 (4-bit Rice
 *     parameters) and 1 (5-bit), escape partitions with raw n-bit samples;
 *   - stereo decorrelation left/side, side/right, mid/side;
 *   - byte padding and CRC-16 (poly 0x8005) over the whole frame.
 * Output: channel-major int32 samples [channels][n] (the integer PCM values).
 * Every structural violation and CRC mismatch is an error (message in err).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t* p;
  size_t n;     /* bytes */
  size_t pos;   /* bit position */
  int bad;      /* read past the end */
} Bits;

static uint32_t get_bits(Bits* b, int k) { /* k <= 32 */
  uint32_t v = 0;
  for (int i = 0; i < k; ++i) {
    const size_t byte = b->pos >> 3;
    if (byte >= b->n) {
      b->bad = 1;
      return 0;
    }
    v = (v << 1) | ((b->p[byte] >> (7 - (b->pos & 7))) & 1u);
    ++b->pos;
  }
  return v;
}

static uint64_t get_bits64(Bits* b, int k) {
  uint64_t v = 0;
  while (k > 0) {
    const int t = k > 32 ? 32 : k;
    v = (v << t) | get_bits(b, t);
    k -= t;
  }
  return v;
}

static int64_t get_signed(Bits* b, int k) {
  if (k == 0) return 0;
  const uint64_t v = get_bits64(b, k);
  return (v >> (k - 1)) & 1u ? (int64_t)(v - (1ull << k)) : (int64_t)v;
}

static uint32_t get_unary(Bits* b) { /* count of 0 bits before a 1 */
  uint32_t q = 0;
  while (!b->bad && get_bits(b, 1) == 0) ++q;
  return q;
}

static uint8_t crc8(const uint8_t* p, size_t n) {
  uint8_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
  }
  return c;
}

static uint16_t crc16(const uint8_t* p, size_t n) {
  uint16_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c ^= (uint16_t)(p[i] << 8);
    for (int k = 0; k < 8; ++k) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x8005 : (c << 1));
  }
  return c;
}

#define FAIL(...)                              \
  do {                                         \
    snprintf(err, (size_t)errlen, __VA_ARGS__); \
    return -1;                                 \
  } while (0)

/* residual of one subframe -> res[order .. bs) */
static int read_residual(Bits* b, int bs, int order, int64_t* res, char* err, int errlen) {
  const uint32_t method = get_bits(b, 2);
  if (method > 1) FAIL("reserved residual coding method %u", method);
  const int pbits = method ? 5 : 4;
  const uint32_t esc = method ? 31u : 15u;
  const int porder = (int)get_bits(b, 4);
  const int parts = 1 << porder;
  if ((bs >> porder) < order || (bs & (parts - 1))) FAIL("bad residual partition order %d", porder);
  int i = order;
  for (int pi = 0; pi < parts; ++pi) {
    const int cnt = (bs >> porder) - (pi == 0 ? order : 0);
    const uint32_t k = get_bits(b, pbits);
    if (k == esc) {
      const int nb = (int)get_bits(b, 5);
      for (int j = 0; j < cnt; ++j) res[i++] = get_signed(b, nb);
    } else {
      for (int j = 0; j < cnt; ++j) {
        const uint64_t q = get_unary(b);
        const uint64_t u = (q << k) | get_bits64(b, (int)k);
        res[i++] = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
      }
    }
    if (b->bad) FAIL("truncated residual");
  }
  return 0;
}

static int read_subframe(Bits* b, int bs, int bps, int64_t* out, char* err, int errlen) {
  if (get_bits(b, 1)) FAIL("subframe padding bit set");
  const uint32_t type = get_bits(b, 6);
  int wasted = 0;
  if (get_bits(b, 1)) wasted = (int)get_unary(b) + 1;
  if (wasted >= bps) FAIL("wasted bits %d >= sample size %d", wasted, bps);
  const int sb = bps - wasted;
  if (type == 0) { /* CONSTANT */
    const int64_t v = get_signed(b, sb);
    for (int i = 0; i < bs; ++i) out[i] = v;
  } else if (type == 1) { /* VERBATIM */
    for (int i = 0; i < bs; ++i) out[i] = get_signed(b, sb);
  } else if (type >= 8 && type <= 12) { /* FIXED */
    const int order = (int)type - 8;
    if (order > bs) FAIL("fixed order %d > block size %d", order, bs);
    for (int i = 0; i < order; ++i) out[i] = get_signed(b, sb);
    if (read_residual(b, bs, order, out, err, errlen)) return -1;
    for (int i = order; i < bs; ++i) {
      int64_t pred = 0;
      switch (order) {
        case 1: pred = out[i - 1]; break;
        case 2: pred = 2 * out[i - 1] - out[i - 2]; break;
        case 3: pred = 3 * out[i - 1] - 3 * out[i - 2] + out[i - 3]; break;
        case 4: pred = 4 * out[i - 1] - 6 * out[i - 2] + 4 * out[i - 3] - out[i - 4]; break;
        default: break;
      }
      out[i] += pred;
    }
  } else if (type >= 32) { /* LPC */
    const int order = (int)(type & 31) + 1;
    if (order > bs) FAIL("lpc order %d > block size %d", order, bs);
    for (int i = 0; i < order; ++i) out[i] = get_signed(b, sb);
    const int prec = (int)get_bits(b, 4) + 1;
    if (prec == 16) FAIL("invalid lpc coefficient precision");
    const int shift = (int)get_signed(b, 5);
    if (shift < 0) FAIL("negative lpc shift %d", shift);
    int64_t coef[32];
    for (int j = 0; j < order; ++j) coef[j] = get_signed(b, prec);
    if (read_residual(b, bs, order, out, err, errlen)) return -1;
    for (int i = order; i < bs; ++i) {
      int64_t s = 0;
      for (int j = 0; j < order; ++j) s += coef[j] * out[i - 1 - j];
      out[i] += s >> shift;
    }
  } else {
    FAIL("reserved subframe type %u", type);
  }
  if (b->bad) FAIL("truncated subframe");
  if (wasted)
    for (int i = 0; i < bs; ++i) out[i] = (int64_t)((uint64_t)out[i] << wasted);
  return 0;
}

static int read_utf8_number(Bits* b, uint64_t* v) {
  const uint32_t c = get_bits(b, 8);
  int extra;
  uint64_t x;
  if (!(c & 0x80)) {
    *v = c;
    return 0;
  }
  if ((c & 0xE0) == 0xC0) { extra = 1; x = c & 0x1F; }
  else if ((c & 0xF0) == 0xE0) { extra = 2; x = c & 0x0F; }
  else if ((c & 0xF8) == 0xF0) { extra = 3; x = c & 0x07; }
  else if ((c & 0xFC) == 0xF8) { extra = 4; x = c & 0x03; }
  else if ((c & 0xFE) == 0xFC) { extra = 5; x = c & 0x01; }
  else if (c == 0xFE) { extra = 6; x = 0; }
  else return -1;
  for (int i = 0; i < extra; ++i) {
    const uint32_t d = get_bits(b, 8);
    if ((d & 0xC0) != 0x80) return -1;
    x = (x << 6) | (d & 0x3F);
  }
  *v = x;
  return 0;
}

/* Decodes a whole FLAC stream.  On success *out = malloc'd [channels][n] int32
 * (free with wsp_flac_free), returns 0. */
int wsp_flac_decode(const uint8_t* data, size_t n, int32_t** out, int* channels, int* sample_rate, int* bits,
                    int64_t* n_samples, char* err, int errlen) {
  *out = NULL;
  size_t pos = 0;
  /* a leading ID3v2 tag ("ID3", version, flags, syncsafe 28-bit size; a footer
   * flag adds 10 bytes), as common decoders tolerate */
  if (n >= 10 && memcmp(data, "ID3", 3) == 0) {
    const size_t sz = ((size_t)(data[6] & 0x7F) << 21) | ((size_t)(data[7] & 0x7F) << 14) |
                      ((size_t)(data[8] & 0x7F) << 7) | (size_t)(data[9] & 0x7F);
    pos = 10 + sz + ((data[5] & 0x10) ? 10 : 0);
  }
  if (pos + 4 > n || memcmp(data + pos, "fLaC", 4) != 0) FAIL("not a FLAC stream (no fLaC marker)");
  pos += 4;
  int have_info = 0, last = 0;
  int si_rate = 0, si_ch = 0, si_bps = 0, si_maxbs = 0;
  uint64_t si_total = 0;
  while (!last) {
    if (pos + 4 > n) FAIL("truncated metadata");
    last = data[pos] >> 7;
    const int type = data[pos] & 0x7F;
    const size_t len = ((size_t)data[pos + 1] << 16) | ((size_t)data[pos + 2] << 8) | data[pos + 3];
    pos += 4;
    if (pos + len > n) FAIL("truncated metadata block");
    if (type == 0) {
      if (len < 34) FAIL("short STREAMINFO");
      Bits b = {data + pos, len, 0, 0};
      get_bits(&b, 16); /* min block size */
      si_maxbs = (int)get_bits(&b, 16);
      get_bits(&b, 24);
      get_bits(&b, 24);
      si_rate = (int)get_bits(&b, 20);
      si_ch = (int)get_bits(&b, 3) + 1;
      si_bps = (int)get_bits(&b, 5) + 1;
      si_total = get_bits64(&b, 36);
      have_info = 1;
    } else if (type == 127) {
      FAIL("invalid metadata block type");
    }
    pos += len;
  }
  if (!have_info) FAIL("missing STREAMINFO");
  size_t cap = si_total ? (size_t)si_total : (size_t)(si_maxbs > 0 ? si_maxbs : 4096) * 16;
  int32_t* pcm = (int32_t*)malloc(cap * (size_t)si_ch * sizeof(int32_t));
  int64_t* sub = (int64_t*)malloc((size_t)65536 * 8 * sizeof(int64_t));
  if (!pcm || !sub) {
    free(pcm);
    free(sub);
    FAIL("out of memory");
  }
  size_t done = 0;
  int rate = si_rate, bps = si_bps, rc = 0;
  while (pos < n) {
    /* a trailing ID3v1 tag ("TAG" + 125 bytes), or padding after the last frame
     * once STREAMINFO's sample count is decoded, ends the stream */
    if (n - pos >= 3 && memcmp(data + pos, "TAG", 3) == 0) break;
    if (si_total && done >= si_total) break;
    const size_t f0 = pos;
    Bits b = {data, n, pos * 8, 0};
    if (get_bits(&b, 14) != 0x3FFE) { snprintf(err, (size_t)errlen, "lost frame sync at byte %zu", pos); rc = -1; break; }
    if (get_bits(&b, 1)) { snprintf(err, (size_t)errlen, "reserved frame header bit set"); rc = -1; break; }
    const int variable = (int)get_bits(&b, 1);
    const uint32_t bsc = get_bits(&b, 4), src = get_bits(&b, 4), chc = get_bits(&b, 4), ssc = get_bits(&b, 3);
    if (get_bits(&b, 1)) { snprintf(err, (size_t)errlen, "reserved frame header bit set"); rc = -1; break; }
    uint64_t num;
    if (read_utf8_number(&b, &num)) { snprintf(err, (size_t)errlen, "bad frame/sample number"); rc = -1; break; }
    (void)variable;
    int bs;
    if (bsc == 0) { snprintf(err, (size_t)errlen, "reserved block size code"); rc = -1; break; }
    else if (bsc == 1) bs = 192;
    else if (bsc <= 5) bs = 576 << (bsc - 2);
    else if (bsc == 6) bs = (int)get_bits(&b, 8) + 1;
    else if (bsc == 7) bs = (int)get_bits(&b, 16) + 1;
    else bs = 256 << (bsc - 8);
    static const int rates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};
    int fr = si_rate;
    if (src >= 1 && src <= 11) fr = rates[src];
    else if (src == 12) fr = (int)get_bits(&b, 8) * 1000;
    else if (src == 13) fr = (int)get_bits(&b, 16);
    else if (src == 14) fr = (int)get_bits(&b, 16) * 10;
    else if (src == 15) { snprintf(err, (size_t)errlen, "invalid sample rate code"); rc = -1; break; }
    static const int sizes[8] = {0, 8, 12, -1, 16, 20, 24, 32};
    int fb = ssc ? sizes[ssc] : si_bps;
    if (fb < 0) { snprintf(err, (size_t)errlen, "reserved sample size code"); rc = -1; break; }
    int nch;
    if (chc <= 7) nch = (int)chc + 1;
    else if (chc <= 10) nch = 2;
    else { snprintf(err, (size_t)errlen, "reserved channel assignment %u", chc); rc = -1; break; }
    if (b.bad || (b.pos & 7)) { snprintf(err, (size_t)errlen, "truncated frame header"); rc = -1; break; }
    const size_t hend = b.pos >> 3;
    if (hend >= n || crc8(data + f0, hend - f0) != data[hend]) { snprintf(err, (size_t)errlen, "frame header CRC-8 mismatch at byte %zu", f0); rc = -1; break; }
    b.pos += 8;
    if (nch != si_ch) { snprintf(err, (size_t)errlen, "channel count changes mid-stream"); rc = -1; break; }
    if (bs > 65536) { snprintf(err, (size_t)errlen, "block size %d too large", bs); rc = -1; break; }
    rate = fr;
    bps = fb;
    for (int c = 0; c < nch; ++c) {
      int sbps = fb;
      if ((chc == 8 && c == 1) || (chc == 9 && c == 0) || (chc == 10 && c == 1)) sbps += 1; /* side channel */
      if (read_subframe(&b, bs, sbps, sub + (size_t)c * 65536, err, errlen)) { rc = -1; break; }
    }
    if (rc) break;
    if (b.pos & 7) b.pos += 8 - (b.pos & 7); /* zero padding to the byte boundary */
    const size_t fend = b.pos >> 3;
    if (fend + 2 > n) { snprintf(err, (size_t)errlen, "truncated frame footer"); rc = -1; break; }
    const uint16_t want = (uint16_t)((data[fend] << 8) | data[fend + 1]);
    if (crc16(data + f0, fend - f0) != want) { snprintf(err, (size_t)errlen, "frame CRC-16 mismatch at byte %zu", f0); rc = -1; break; }
    pos = fend + 2;
    int64_t* s0 = sub;
    int64_t* s1 = sub + 65536;
    for (int i = 0; i < bs && nch == 2 && chc >= 8; ++i) {
      int64_t l, r;
      if (chc == 8) { l = s0[i]; r = s0[i] - s1[i]; }            /* left / side */
      else if (chc == 9) { r = s1[i]; l = s0[i] + s1[i]; }       /* side / right */
      else { const int64_t m = (s0[i] * 2) | (s1[i] & 1); l = (m + s1[i]) >> 1; r = (m - s1[i]) >> 1; } /* mid / side */
      s0[i] = l;
      s1[i] = r;
    }
    if (done + (size_t)bs > cap) {
      size_t ncap = (done + (size_t)bs) * 2;
      int32_t* np = (int32_t*)malloc(ncap * (size_t)nch * sizeof(int32_t));
      if (!np) { snprintf(err, (size_t)errlen, "out of memory"); rc = -1; break; }
      for (int c = 0; c < nch; ++c) memcpy(np + (size_t)c * ncap, pcm + (size_t)c * cap, done * sizeof(int32_t));
      free(pcm);
      pcm = np;
      cap = ncap;
    }
    for (int c = 0; c < nch; ++c)
      for (int i = 0; i < bs; ++i) pcm[(size_t)c * cap + done + i] = (int32_t)sub[(size_t)c * 65536 + i];
    done += (size_t)bs;
  }
  free(sub);
  if (rc) {
    free(pcm);
    return -1;
  }
  if (si_total && done != si_total) {
    free(pcm);
    FAIL("decoded %zu samples, STREAMINFO says %llu", done, (unsigned long long)si_total);
  }
  /* compact to [channels][done] */
  if (cap != done)
    for (int c = 1; c < si_ch; ++c) memmove(pcm + (size_t)c * done, pcm + (size_t)c * cap, done * sizeof(int32_t));
  *out = pcm;
  *channels = si_ch;
  *sample_rate = rate;
  *bits = bps;
  *n_samples = (int64_t)done;
  return 0;
}

void wsp_flac_free(int32_t* p) { free(p); }
