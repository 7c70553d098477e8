// libsuta_audio.so: FLAC decoder from the format specification (RFC 9639), host code.
// Replaces torchaudio.load for .flac files (reference data.py:15, corpus/librispeech.py:30).
// See include/suta_audio.h for the contract.
#include "../../include/suta_audio.h"

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char* msg) {
    g_err = msg;
    return code;
}

// ---------------------------------------------------------------------------------------------
// CRCs (RFC 9639 9.1.8 / 9.3): CRC-8 poly x^8+x^2+x+1, CRC-16 poly x^16+x^15+x^2+1, MSB first, init 0.
// ---------------------------------------------------------------------------------------------
struct CrcTables {
    uint8_t c8[256];
    uint16_t c16[256];
    CrcTables() {
        for (int i = 0; i < 256; ++i) {
            uint8_t c = (uint8_t)i;
            for (int b = 0; b < 8; ++b) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
            c8[i] = c;
            uint16_t d = (uint16_t)(i << 8);
            for (int b = 0; b < 8; ++b) d = (uint16_t)((d & 0x8000) ? (d << 1) ^ 0x8005 : (d << 1));
            c16[i] = d;
        }
    }
};
const CrcTables& crc() {
    static const CrcTables t;
    return t;
}
uint8_t crc8(const uint8_t* p, size_t n) {
    uint8_t c = 0;
    for (size_t i = 0; i < n; ++i) c = crc().c8[c ^ p[i]];
    return c;
}
uint16_t crc16(const uint8_t* p, size_t n) {
    uint16_t c = 0;
    for (size_t i = 0; i < n; ++i) c = (uint16_t)((c << 8) ^ crc().c16[(c >> 8) ^ p[i]]);
    return c;
}

// ---------------------------------------------------------------------------------------------
// MSB-first bit reader over [p, end) with a 64-bit cache.
// ---------------------------------------------------------------------------------------------
struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t cache = 0;  // valid bits left-aligned
    int n = 0;           // number of valid bits in cache
    bool overrun = false;

    Bits(const uint8_t* b, const uint8_t* e) : p(b), end(e) {}

    // position in bytes of the next unread bit's byte (only meaningful when byte aligned)
    const uint8_t* byte_pos() const { return p - n / 8; }
    uint64_t bits_left() const { return (uint64_t)(end - p) * 8 + (uint64_t)n; }

    uint32_t get(int k) {  // k <= 32
        if (k == 0) return 0;
        if (n < k) fill(k);
        if (n < k) { overrun = true; return 0; }
        uint32_t v = (uint32_t)(cache >> (64 - k));
        cache <<= k;
        n -= k;
        return v;
    }
    void fill(int need) {
        while (n < need && n <= 56) {
            if (p >= end) return;
            cache |= (uint64_t)(*p++) << (56 - n);
            n += 8;
        }
    }
    int32_t get_signed(int k) {  // two's complement field of k bits (k <= 32)
        if (k == 0) return 0;
        uint32_t v = get(k);
        if (k < 32 && (v >> (k - 1))) v |= ~0u << k;
        return (int32_t)v;
    }
    int64_t get_signed_wide(int k) {  // k <= 33 (side channel of a 32-bit stream)
        if (k <= 32) return get_signed(k);
        int64_t hi = get_signed(k - 32);
        return (int64_t)((uint64_t)hi << 32) | get(32);
    }
    uint32_t unary() {  // count zeros up to the next 1 (consumes the 1)
        uint32_t q = 0;
        for (;;) {
            if (n == 0) fill(8);
            if (n == 0) { overrun = true; return q; }
            if (cache == 0) { q += (uint32_t)n; cache = 0; n = 0; continue; }
            int lz = __builtin_clzll(cache);
            if (lz >= n) { q += (uint32_t)n; cache = 0; n = 0; continue; }
            q += (uint32_t)lz;
            cache <<= (lz + 1);
            n -= lz + 1;
            return q;
        }
    }
    void align() { int r = n & 7; cache <<= r; n -= r; }
};

struct StreamInfo {
    uint32_t min_block = 0, max_block = 0, rate = 0, channels = 0, bps = 0;
    uint64_t total = 0;
};

int parse_header(const uint8_t* buf, int64_t len, StreamInfo* si, int64_t* frames_at) {
    int64_t o = 0;
    if (len >= 10 && buf[0] == 'I' && buf[1] == 'D' && buf[2] == '3') {  // ID3v2 tag before the stream
        int64_t sz = ((int64_t)(buf[6] & 0x7f) << 21) | ((buf[7] & 0x7f) << 14) | ((buf[8] & 0x7f) << 7) |
                     (buf[9] & 0x7f);
        o = 10 + sz + ((buf[5] & 0x10) ? 10 : 0);
    }
    if (len < o + 4 || memcmp(buf + o, "fLaC", 4) != 0) return fail(SUTA_AUDIO_ERR_FORMAT, "no fLaC marker");
    o += 4;
    bool have_si = false;
    for (;;) {
        if (o + 4 > len) return fail(SUTA_AUDIO_ERR_TRUNC, "truncated metadata block header");
        int last = buf[o] >> 7, type = buf[o] & 0x7f;
        int64_t bl = ((int64_t)buf[o + 1] << 16) | (buf[o + 2] << 8) | buf[o + 3];
        o += 4;
        if (o + bl > len) return fail(SUTA_AUDIO_ERR_TRUNC, "truncated metadata block");
        if (type == 127) return fail(SUTA_AUDIO_ERR_FORMAT, "invalid metadata block type 127");
        if (type == 0) {
            if (bl < 34) return fail(SUTA_AUDIO_ERR_FORMAT, "short STREAMINFO");
            Bits b(buf + o, buf + o + bl);
            si->min_block = b.get(16);
            si->max_block = b.get(16);
            b.get(24);
            b.get(24);
            si->rate = b.get(20);
            si->channels = b.get(3) + 1;
            si->bps = b.get(5) + 1;
            uint64_t hi = b.get(4);
            si->total = (hi << 32) | b.get(32);
            have_si = true;
        }
        o += bl;
        if (last) break;
    }
    if (!have_si) return fail(SUTA_AUDIO_ERR_FORMAT, "first metadata block is not STREAMINFO");
    *frames_at = o;
    return SUTA_AUDIO_OK;
}

// residual coding (RFC 9639 9.2.7): res[0..bs-order)
int read_residual(Bits& b, int bs, int order, int32_t* res) {
    uint32_t method = b.get(2);
    if (method > 1) return fail(SUTA_AUDIO_ERR_FORMAT, "reserved residual coding method");
    int pbits = method == 0 ? 4 : 5;
    uint32_t escape = method == 0 ? 15u : 31u;
    int porder = (int)b.get(4);
    int parts = 1 << porder;
    if ((bs >> porder) << porder != bs) return fail(SUTA_AUDIO_ERR_FORMAT, "block size not divisible by partitions");
    int psz = bs >> porder;
    if (psz < order) return fail(SUTA_AUDIO_ERR_FORMAT, "first partition shorter than predictor order");
    int k = 0;
    for (int pi = 0; pi < parts; ++pi) {
        int cnt = pi == 0 ? psz - order : psz;
        uint32_t param = b.get(pbits);
        if (param == escape) {
            int nb = (int)b.get(5);
            for (int i = 0; i < cnt; ++i) res[k++] = b.get_signed(nb);
        } else {
            for (int i = 0; i < cnt; ++i) {
                uint32_t q = b.unary();
                uint32_t u = (q << param) | b.get((int)param);
                res[k++] = (int32_t)(u >> 1) ^ -(int32_t)(u & 1);
            }
        }
        if (b.overrun) return fail(SUTA_AUDIO_ERR_TRUNC, "stream ends inside a residual");
    }
    return SUTA_AUDIO_OK;
}

// one subframe into s[0..bs) (int64 so side channels of 32-bit streams and LPC sums stay exact)
int read_subframe(Bits& b, int bs, int bps, int64_t* s, std::vector<int32_t>& res) {
    if (b.get(1) != 0) return fail(SUTA_AUDIO_ERR_FORMAT, "subframe padding bit set");
    uint32_t type = b.get(6);
    int wasted = 0;
    if (b.get(1)) wasted = (int)b.unary() + 1;
    if (wasted >= bps) return fail(SUTA_AUDIO_ERR_FORMAT, "wasted bits exceed sample size");
    int eb = bps - wasted;
    if (type == 0) {  // CONSTANT
        int64_t v = b.get_signed_wide(eb);
        for (int i = 0; i < bs; ++i) s[i] = v;
    } else if (type == 1) {  // VERBATIM
        for (int i = 0; i < bs; ++i) s[i] = b.get_signed_wide(eb);
    } else if (type >= 8 && type <= 12) {  // FIXED, order 0..4
        int order = (int)type - 8;
        if (order > bs) return fail(SUTA_AUDIO_ERR_FORMAT, "fixed order exceeds block size");
        for (int i = 0; i < order; ++i) s[i] = b.get_signed_wide(eb);
        res.resize(bs);
        int st = read_residual(b, bs, order, res.data());
        if (st) return st;
        const int32_t* r = res.data();
        switch (order) {
            case 0: for (int i = 0; i < bs; ++i) s[i] = r[i]; break;
            case 1: for (int i = 1; i < bs; ++i) s[i] = s[i - 1] + r[i - 1]; break;
            case 2: for (int i = 2; i < bs; ++i) s[i] = 2 * s[i - 1] - s[i - 2] + r[i - 2]; break;
            case 3: for (int i = 3; i < bs; ++i) s[i] = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3] + r[i - 3]; break;
            case 4:
                for (int i = 4; i < bs; ++i) s[i] = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4] + r[i - 4];
                break;
        }
    } else if (type >= 32) {  // LPC, order 1..32
        int order = (int)(type & 31) + 1;
        if (order > bs) return fail(SUTA_AUDIO_ERR_FORMAT, "LPC order exceeds block size");
        for (int i = 0; i < order; ++i) s[i] = b.get_signed_wide(eb);
        uint32_t prec = b.get(4);
        if (prec == 15) return fail(SUTA_AUDIO_ERR_FORMAT, "invalid LPC coefficient precision");
        int precision = (int)prec + 1;
        int shift = b.get_signed(5);
        if (shift < 0) return fail(SUTA_AUDIO_ERR_FORMAT, "negative LPC shift");
        int64_t coef[32];
        for (int i = 0; i < order; ++i) coef[i] = b.get_signed(precision);
        res.resize(bs);
        int st = read_residual(b, bs, order, res.data());
        if (st) return st;
        for (int i = order; i < bs; ++i) {
            int64_t acc = 0;
            for (int j = 0; j < order; ++j) acc += coef[j] * s[i - 1 - j];
            s[i] = (acc >> shift) + res[i - order];
        }
    } else {
        return fail(SUTA_AUDIO_ERR_FORMAT, "reserved subframe type");
    }
    if (b.overrun) return fail(SUTA_AUDIO_ERR_TRUNC, "stream ends inside a subframe");
    if (wasted)
        for (int i = 0; i < bs; ++i) s[i] = s[i] * ((int64_t)1 << wasted);
    return SUTA_AUDIO_OK;
}

const int kBps[8] = {0, 8, 12, -1, 16, 20, 24, 32};

}  // namespace

// shared with mp3.cpp (the other decoder of libsuta_audio.so): one per-thread message for both
namespace suta_audio_internal {
void set_error(const char* msg) { g_err = msg; }
}  // namespace suta_audio_internal

extern "C" {

int32_t suta_flac_info(const uint8_t* buf, int64_t len, int32_t* sample_rate, int32_t* channels,
                       int32_t* bits_per_sample, int64_t* total_samples) {
    if (!buf || len <= 0) return fail(SUTA_AUDIO_ERR_FORMAT, "empty buffer");
    StreamInfo si;
    int64_t at = 0;
    int st = parse_header(buf, len, &si, &at);
    if (st) return st;
    if (sample_rate) *sample_rate = (int32_t)si.rate;
    if (channels) *channels = (int32_t)si.channels;
    if (bits_per_sample) *bits_per_sample = (int32_t)si.bps;
    if (total_samples) *total_samples = (int64_t)si.total;
    return SUTA_AUDIO_OK;
}

int32_t suta_flac_decode(const uint8_t* buf, int64_t len, float* out, int64_t out_capacity, int32_t verify_crc,
                         int64_t* n_out) {
    if (!buf || len <= 0 || !n_out) return fail(SUTA_AUDIO_ERR_FORMAT, "empty buffer");
    StreamInfo si;
    int64_t at = 0;
    int st = parse_header(buf, len, &si, &at);
    if (st) return st;
    if (si.total && (int64_t)si.total > out_capacity) {
        *n_out = (int64_t)si.total;
        return fail(SUTA_AUDIO_ERR_SPACE, "output capacity below STREAMINFO total samples");
    }
    const int C = (int)si.channels;
    std::vector<int64_t> chan[8];
    std::vector<int32_t> res;
    int64_t done = 0;
    bool space_short = false;
    const uint8_t* end = buf + len;
    const uint8_t* p = buf + at;
    while (p + 2 <= end) {
        if (!(p[0] == 0xFF && (p[1] & 0xFE) == 0xF8)) {
            // trailing garbage / tags after the last frame: stop if we already decoded the total
            if (si.total && done >= (int64_t)si.total) break;
            return fail(SUTA_AUDIO_ERR_FORMAT, "frame sync code expected");
        }
        const uint8_t* frame = p;
        Bits b(p, end);
        b.get(15);
        b.get(1);  // blocking strategy: the coded number is only used for seeking
        uint32_t bs_code = b.get(4), sr_code = b.get(4), ch_code = b.get(4), ss_code = b.get(3);
        if (b.get(1)) return fail(SUTA_AUDIO_ERR_FORMAT, "frame header reserved bit set");
        // UTF-8-style coded frame / sample number
        uint32_t first = b.get(8);
        int extra = 0;
        if (first & 0x80) {
            if ((first & 0xE0) == 0xC0) extra = 1;
            else if ((first & 0xF0) == 0xE0) extra = 2;
            else if ((first & 0xF8) == 0xF0) extra = 3;
            else if ((first & 0xFC) == 0xF8) extra = 4;
            else if ((first & 0xFE) == 0xFC) extra = 5;
            else if (first == 0xFE) extra = 6;
            else return fail(SUTA_AUDIO_ERR_FORMAT, "invalid coded frame number");
        }
        for (int i = 0; i < extra; ++i)
            if ((b.get(8) & 0xC0) != 0x80) return fail(SUTA_AUDIO_ERR_FORMAT, "invalid coded frame number");
        int bs;
        if (bs_code == 0) return fail(SUTA_AUDIO_ERR_FORMAT, "reserved block size code");
        else if (bs_code == 1) bs = 192;
        else if (bs_code <= 5) bs = 576 << (bs_code - 2);
        else if (bs_code == 6) bs = (int)b.get(8) + 1;
        else if (bs_code == 7) bs = (int)b.get(16) + 1;
        else bs = 256 << (bs_code - 8);
        if (sr_code == 12) b.get(8);
        else if (sr_code == 13 || sr_code == 14) b.get(16);
        else if (sr_code == 15) return fail(SUTA_AUDIO_ERR_FORMAT, "invalid sample rate code");
        int bps = ss_code == 0 ? (int)si.bps : kBps[ss_code];
        if (bps < 0) return fail(SUTA_AUDIO_ERR_FORMAT, "reserved sample size code");
        int nch;
        if (ch_code <= 7) nch = (int)ch_code + 1;
        else if (ch_code <= 10) nch = 2;
        else return fail(SUTA_AUDIO_ERR_FORMAT, "reserved channel assignment");
        if (nch != C) return fail(SUTA_AUDIO_ERR_FORMAT, "frame channel count differs from STREAMINFO");
        if (b.overrun) return fail(SUTA_AUDIO_ERR_TRUNC, "stream ends inside a frame header");
        uint32_t hcrc = b.get(8);
        const uint8_t* hdr_end = b.byte_pos();  // header is byte aligned here
        if (verify_crc && crc8(frame, (size_t)(hdr_end - frame - 1)) != hcrc)
            return fail(SUTA_AUDIO_ERR_CRC, "frame header CRC-8 mismatch");
        for (int c = 0; c < C; ++c) {
            chan[c].resize(bs);
            int sbps = bps;
            if ((ch_code == 8 && c == 1) || (ch_code == 9 && c == 0) || (ch_code == 10 && c == 1)) sbps = bps + 1;
            st = read_subframe(b, bs, sbps, chan[c].data(), res);
            if (st) return st;
        }
        b.align();
        uint32_t fcrc = b.get(16);
        if (b.overrun) return fail(SUTA_AUDIO_ERR_TRUNC, "stream ends inside a frame");
        const uint8_t* fend = b.byte_pos();
        if (verify_crc && crc16(frame, (size_t)(fend - frame - 2)) != fcrc)
            return fail(SUTA_AUDIO_ERR_CRC, "frame CRC-16 mismatch");
        p = fend;
        // inter-channel decorrelation
        if (ch_code == 8) {
            for (int i = 0; i < bs; ++i) chan[1][i] = chan[0][i] - chan[1][i];
        } else if (ch_code == 9) {
            for (int i = 0; i < bs; ++i) chan[0][i] = chan[0][i] + chan[1][i];
        } else if (ch_code == 10) {
            for (int i = 0; i < bs; ++i) {
                int64_t side = chan[1][i];
                int64_t mid = (chan[0][i] * 2) | (side & 1);
                chan[0][i] = (mid + side) >> 1;
                chan[1][i] = (mid - side) >> 1;
            }
        }
        const float scale = 1.0f / (float)((int64_t)1 << (bps - 1));
        int64_t room = out_capacity - done;
        int take = (int64_t)bs <= room ? bs : (int)(room > 0 ? room : 0);
        if (take < bs) space_short = true;
        if (out)
            for (int c = 0; c < C; ++c) {
                float* o = out + (int64_t)c * out_capacity + done;
                const int64_t* s = chan[c].data();
                for (int i = 0; i < take; ++i) o[i] = (float)s[i] * scale;
            }
        done += bs;
    }
    *n_out = done;
    if (space_short) return fail(SUTA_AUDIO_ERR_SPACE, "output capacity below decoded samples");
    if (si.total && done != (int64_t)si.total) return fail(SUTA_AUDIO_ERR_TRUNC, "decoded fewer samples than STREAMINFO states");
    return SUTA_AUDIO_OK;
}

const char* suta_audio_last_error(void) { return g_err.c_str(); }

}  // extern "C"
