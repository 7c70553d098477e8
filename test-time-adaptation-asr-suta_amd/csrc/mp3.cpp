// libsuta_audio.so: MPEG-1 / MPEG-2 / MPEG-2.5 Audio Layer III decoder, host code, written from the
// format specification (ISO/IEC 11172-3 section 2.4 and Annex A/B, ISO/IEC 13818-3 for the low sampling
// frequencies).  Replaces torchaudio.load for the CommonVoice clips (reference corpus/commonvoice.py:32-38 reads
// clips/*.mp3, reference data.py:15 loads them).  See include/suta_audio.h for the contract.
//
// Normative tables the decoder cannot compute (Huffman code tables B.7, synthesis window B.3) are in
// mp3_tables.h (generated and checked by tools/mp3_tables.py); band tables, count1 tables, pretab and the
// antialias coefficients are typed below.  Everything else (IMDCT, windows, polyphase matrixing, requantisation,
// stereo ratios) is computed from the formulas of the standard, in double precision.
//
// Decoder delay and gapless trimming follow FFmpeg (the MP3 backend of torchaudio; libavformat mp3dec.c
// mp3_parse_info_tag and the demuxer's discard window): the Xing / Info frame is not decoded; when it carries an
// encoder tag (LAME / Lavc / Lavf) the first enc_delay + 529 samples are dropped, and only when the Xing frames
// field is present (flags & 1, count F != 0) the decoded positions [F * spf - enc_padding + 529, F * spf) are dropped
// from every frame (packet) that overlaps them -- measured from the Xing count, not from the frames this scan finds,
// so a truncated stream keeps its tail; without a tag every decoded sample is returned.
#include "../../include/suta_audio.h"
#include "mp3_tables.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

namespace suta_audio_internal {
void set_error(const char* msg);
}

namespace {

int fail(int code, const char* msg) {
    suta_audio_internal::set_error(msg);
    return code;
}

// ---------------------------------------------------------------------------------------------
// Tables typed from the standard
// ---------------------------------------------------------------------------------------------
// Annex B.8 scale-factor band boundaries: index = sampling-frequency index 0..8
// (MPEG-1 44.1 / 48 / 32 kHz, MPEG-2 22.05 / 24 / 16 kHz, MPEG-2.5 11.025 / 12 / 8 kHz)
const int kSfbLong[9][23] = {
    {0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576},
    {0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576},
    {0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576},
    {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
    {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 114, 136, 162, 194, 232, 278, 330, 394, 464, 540, 576},
    {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
    {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
    {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
    {0, 12, 24, 36, 48, 60, 72, 88, 108, 132, 160, 192, 232, 280, 336, 400, 476, 566, 568, 570, 572, 574, 576},
};
const int kSfbShort[9][14] = {
    {0, 4, 8, 12, 16, 22, 30, 40, 52, 66, 84, 106, 136, 192},
    {0, 4, 8, 12, 16, 22, 28, 38, 50, 64, 80, 100, 126, 192},
    {0, 4, 8, 12, 16, 22, 30, 42, 58, 78, 104, 138, 180, 192},
    {0, 4, 8, 12, 18, 24, 32, 42, 56, 74, 100, 132, 174, 192},
    {0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 136, 180, 192},
    {0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192},
    {0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192},
    {0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192},
    {0, 8, 16, 24, 36, 52, 72, 96, 124, 160, 162, 164, 166, 192},
};
const int kPretab[22] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 2, 2, 3, 3, 3, 2, 0, 0};
const double kAliasC[8] = {-0.6, -0.535, -0.33, -0.185, -0.095, -0.041, -0.0142, -0.0037};
// 2.4.2.7 scalefac_compress (MPEG-1): slen1, slen2
const int kSlen[2][16] = {{0, 0, 0, 0, 3, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4},
                          {0, 1, 2, 3, 0, 1, 2, 3, 1, 2, 3, 1, 2, 3, 2, 3}};
// ISO/IEC 13818-3 2.4.3.2 nr_of_sfb[table][block: long, short, mixed][partition]
const int kNrSfb[6][3][4] = {
    {{6, 5, 5, 5}, {9, 9, 9, 9}, {6, 9, 9, 9}},    {{6, 5, 7, 3}, {9, 9, 12, 6}, {6, 9, 12, 6}},
    {{11, 10, 0, 0}, {18, 18, 0, 0}, {15, 18, 0, 0}}, {{7, 7, 7, 0}, {12, 12, 12, 0}, {6, 15, 12, 0}},
    {{6, 6, 6, 3}, {12, 9, 9, 6}, {6, 12, 9, 6}},  {{8, 8, 5, 0}, {15, 12, 9, 0}, {6, 18, 9, 0}}};
// count1 table A (Table B.7 "A"): value = v*8 + w*4 + x*2 + y; table B is 4 bits, code = 15 - value
const uint8_t kQuadLen[16] = {1, 4, 4, 5, 4, 6, 5, 6, 4, 5, 5, 6, 5, 6, 6, 6};
const uint16_t kQuadCod[16] = {1, 5, 4, 5, 6, 5, 4, 4, 7, 3, 6, 0, 7, 2, 3, 1};
const int kBitrate[2][15] = {{0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320},
                             {0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160}};
const int kRate[9] = {44100, 48000, 32000, 22050, 24000, 16000, 11025, 12000, 8000};

// ---------------------------------------------------------------------------------------------
// Huffman decoding trees and the computed tables (built once; C++11 static init is thread-safe)
// ---------------------------------------------------------------------------------------------
struct Tree {
    // node i has children node[2i], node[2i+1]; a child >= 0 is a node index, < 0 a leaf -(value + 1)
    std::vector<int32_t> node;
    bool build(const uint8_t* len, const uint16_t* cod, int count) {
        node.assign(2, 0);
        for (int v = 0; v < count; ++v) {
            int at = 0;
            for (int b = len[v] - 1; b >= 0; --b) {
                int bit = (cod[v] >> b) & 1;
                int32_t& child = node[2 * at + bit];
                if (b == 0) {
                    if (child != 0) return false;
                    child = -(v + 1);
                } else {
                    if (child < 0) return false;
                    if (child == 0) {
                        child = (int32_t)(node.size() / 2);
                        node.push_back(0);
                        node.push_back(0);
                    }
                    at = node[2 * at + bit];
                }
            }
        }
        return true;
    }
};

struct Tables {
    Tree big[34];  // by table id 0..31 (16..23 -> 16, 24..31 -> 24); [32] = count1 A
    int size[32] = {0};
    int linbits[32] = {0};
    bool ok = true;
    double pow43[8207];
    double D[512];
    double N[64][32];
    double imdct36[36][18], imdct12[12][6];
    double win[4][36], win12[12];
    double cs[8], ca[8];
    Tables() {
        using namespace mp3tab;
        struct Src { int id, n; const uint8_t* l; const uint16_t* c; };
        const Src src[] = {{1, 2, hlen1, hcod1},     {2, 3, hlen2, hcod2},     {3, 3, hlen3, hcod3},
                           {5, 4, hlen5, hcod5},     {6, 4, hlen6, hcod6},     {7, 6, hlen7, hcod7},
                           {8, 6, hlen8, hcod8},     {9, 6, hlen9, hcod9},     {10, 8, hlen10, hcod10},
                           {11, 8, hlen11, hcod11},  {12, 8, hlen12, hcod12},  {13, 16, hlen13, hcod13},
                           {15, 16, hlen15, hcod15}, {16, 16, hlen16, hcod16}, {24, 16, hlen24, hcod24}};
        for (const Src& s : src) {
            ok = ok && big[s.id].build(s.l, s.c, s.n * s.n);
            size[s.id] = s.n;
        }
        const int lb16[8] = {1, 2, 3, 4, 6, 8, 10, 13}, lb24[8] = {4, 5, 6, 7, 8, 9, 11, 13};
        for (int i = 0; i < 8; ++i) {
            size[16 + i] = 16; linbits[16 + i] = lb16[i];
            size[24 + i] = 16; linbits[24 + i] = lb24[i];
        }
        ok = ok && big[32].build(kQuadLen, kQuadCod, 16);
        for (int i = 0; i < 8207; ++i) pow43[i] = std::pow((double)i, 4.0 / 3.0);
        // Table B.3: D[i] = window257[i] / 65536 for i <= 256, D[512 - i] = +-D[i]
        for (int i = 0; i <= 256; ++i) {
            double v = window257[i] / 65536.0;
            D[i] = v;
            if (i > 0) D[512 - i] = (i % 64 == 0) ? v : -v;
        }
        const double pi = 3.14159265358979323846;
        for (int i = 0; i < 64; ++i)
            for (int k = 0; k < 32; ++k) N[i][k] = std::cos((16 + i) * (2 * k + 1) * pi / 64.0);
        for (int i = 0; i < 36; ++i)
            for (int k = 0; k < 18; ++k) imdct36[i][k] = std::cos(pi / 72.0 * (2 * i + 1 + 18) * (2 * k + 1));
        for (int i = 0; i < 12; ++i)
            for (int k = 0; k < 6; ++k) imdct12[i][k] = std::cos(pi / 24.0 * (2 * i + 1 + 6) * (2 * k + 1));
        // 2.4.3.4.10.3 windows of block types 0 (normal), 1 (start), 3 (stop); type 2 uses win12
        for (int i = 0; i < 36; ++i) win[0][i] = std::sin(pi / 36 * (i + 0.5));
        for (int i = 0; i < 36; ++i) {
            win[1][i] = i < 18 ? std::sin(pi / 36 * (i + 0.5))
                      : i < 24 ? 1.0
                      : i < 30 ? std::sin(pi / 12 * (i - 18 + 0.5)) : 0.0;
            win[3][i] = i < 6 ? 0.0
                      : i < 12 ? std::sin(pi / 12 * (i - 6 + 0.5))
                      : i < 18 ? 1.0 : std::sin(pi / 36 * (i + 0.5));
        }
        for (int i = 0; i < 12; ++i) win12[i] = std::sin(pi / 12 * (i + 0.5));
        for (int i = 0; i < 8; ++i) {
            double sq = std::sqrt(1.0 + kAliasC[i] * kAliasC[i]);
            cs[i] = 1.0 / sq;
            ca[i] = kAliasC[i] / sq;
        }
    }
};
const Tables& tabs() {
    static const Tables t;
    return t;
}

// ---------------------------------------------------------------------------------------------
// Frame header (2.4.1.3)
// ---------------------------------------------------------------------------------------------
struct Header {
    int lsf;        // 0 MPEG-1, 1 MPEG-2 / 2.5 (low sampling frequencies: one granule per frame)
    int sfreq;      // 0..8 as kRate
    int crc;        // a 16-bit CRC follows the header
    int bitrate;    // kbit/s
    int padding;
    int mode;       // 0 stereo, 1 joint stereo, 2 dual channel, 3 single channel
    int mode_ext;
    int channels;
    int frame_bytes;
    int side_bytes;
    int granules;
};

bool parse_header(const uint8_t* p, Header* h) {
    if (p[0] != 0xFF || (p[1] & 0xE0) != 0xE0) return false;
    int ver = (p[1] >> 3) & 3;     // 3 MPEG-1, 2 MPEG-2, 0 MPEG-2.5
    int layer = (p[1] >> 1) & 3;   // 1 = Layer III
    if (ver == 1 || layer != 1) return false;
    int bri = p[2] >> 4, sri = (p[2] >> 2) & 3;
    if (bri == 0 || bri == 15 || sri == 3) return false;  // free format is not supported
    h->lsf = ver != 3;
    h->sfreq = (ver == 3 ? 0 : ver == 2 ? 3 : 6) + sri;
    h->crc = !(p[1] & 1);
    h->bitrate = kBitrate[h->lsf][bri];
    h->padding = (p[2] >> 1) & 1;
    h->mode = p[3] >> 6;
    h->mode_ext = (p[3] >> 4) & 3;
    h->channels = h->mode == 3 ? 1 : 2;
    int rate = kRate[h->sfreq];
    h->frame_bytes = (h->lsf ? 72000 : 144000) * h->bitrate / rate + h->padding;
    h->side_bytes = h->lsf ? (h->channels == 1 ? 9 : 17) : (h->channels == 1 ? 17 : 32);
    h->granules = h->lsf ? 1 : 2;
    return h->frame_bytes >= 4 + 2 * h->crc + h->side_bytes;
}

// MSB-first bit reader over a byte range
struct BitReader {
    const uint8_t* p;
    int64_t nbits, pos = 0;
    BitReader(const uint8_t* b, int64_t nbytes) : p(b), nbits(nbytes * 8) {}
    uint32_t get(int k) {
        uint32_t v = 0;
        for (int i = 0; i < k; ++i, ++pos) {
            int bit = pos < nbits ? (p[pos >> 3] >> (7 - (pos & 7))) & 1 : 0;
            v = (v << 1) | (uint32_t)bit;
        }
        return v;
    }
    int bit() { return (int)get(1); }
};

struct Granule {
    int part23, big_values, global_gain, sfc, ws, block_type, mixed;
    int table[3], subblock_gain[3], region0, region1, preflag, sf_scale, count1_table;
};

struct SideInfo {
    int main_data_begin;
    int scfsi[2][4];
    Granule gr[2][2];
};

void read_side_info(BitReader& b, const Header& h, SideInfo* si) {
    std::memset(si, 0, sizeof(*si));
    si->main_data_begin = (int)b.get(h.lsf ? 8 : 9);
    b.get(h.lsf ? (h.channels == 1 ? 1 : 2) : (h.channels == 1 ? 5 : 3));  // private bits
    if (!h.lsf)
        for (int ch = 0; ch < h.channels; ++ch)
            for (int g = 0; g < 4; ++g) si->scfsi[ch][g] = b.bit();
    for (int gr = 0; gr < h.granules; ++gr)
        for (int ch = 0; ch < h.channels; ++ch) {
            Granule& g = si->gr[gr][ch];
            g.part23 = (int)b.get(12);
            g.big_values = (int)b.get(9);
            g.global_gain = (int)b.get(8);
            g.sfc = (int)b.get(h.lsf ? 9 : 4);
            g.ws = b.bit();
            if (g.ws) {
                g.block_type = (int)b.get(2);
                g.mixed = b.bit();
                g.table[0] = (int)b.get(5);
                g.table[1] = (int)b.get(5);
                for (int w = 0; w < 3; ++w) g.subblock_gain[w] = (int)b.get(3);
            } else {
                for (int r = 0; r < 3; ++r) g.table[r] = (int)b.get(5);
                g.region0 = (int)b.get(4);
                g.region1 = (int)b.get(3);
            }
            if (!h.lsf) g.preflag = b.bit();
            g.sf_scale = b.bit();
            g.count1_table = b.bit();
        }
}

// scale factors of one granule / channel: long bands 0..21, short bands [0..12][window]; slen of each band
// (the MPEG-2 intensity-stereo "illegal position" is 2^slen - 1)
struct ScaleFactors {
    int l[22];
    int s[13][3];
    int lslen[22];
    int sslen[13];
};

// ---------------------------------------------------------------------------------------------
// The decoder
// ---------------------------------------------------------------------------------------------
struct Stats {
    int64_t frames = 0, granules = 0, exact = 0, overrun = 0, lost = 0;
};

class Decoder {
   public:
    explicit Decoder(int channels) : nch_(channels) {
        std::memset(overlap_, 0, sizeof(overlap_));
        std::memset(vbuf_, 0, sizeof(vbuf_));
        voff_[0] = voff_[1] = 0;
    }

    // Decode one frame; appends granules * 576 samples per channel to pcm[ch].
    int frame(const uint8_t* f, const Header& h, std::vector<float>* pcm, Stats* st, bool strict) {
        int hdr = 4 + 2 * h.crc;
        BitReader sb(f + hdr, h.side_bytes);
        SideInfo si;
        read_side_info(sb, h, &si);
        const uint8_t* md = f + hdr + h.side_bytes;
        int md_len = h.frame_bytes - hdr - h.side_bytes;
        int64_t have = (int64_t)res_.size();
        bool lost = si.main_data_begin > have;
        int64_t start = have - si.main_data_begin;
        res_.insert(res_.end(), md, md + md_len);
        ++st->frames;
        if (lost) {  // bit reservoir not available (stream cut): the frame's granules are silent
            ++st->lost;
            for (int gr = 0; gr < h.granules; ++gr)
                for (int ch = 0; ch < nch_; ++ch) pcm[ch].insert(pcm[ch].end(), 576, 0.0f);
            trim_reservoir();
            return 0;
        }
        BitReader br(res_.data() + start, (int64_t)res_.size() - start);
        ScaleFactors sf[2][2];
        for (int gr = 0; gr < h.granules; ++gr) {
            double xr[2][576];
            int nonzero[2];
            for (int ch = 0; ch < h.channels; ++ch) {
                Granule& g = si.gr[gr][ch];
                if (g.ws && g.block_type == 0) return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: reserved block type 0 with window switching");
                if (g.big_values > 288) return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: big_values > 288");
                int64_t p0 = br.pos;
                if (h.lsf) read_sf_lsf(br, h, g, ch, &sf[gr][ch]);
                else read_sf_mpeg1(br, g, si.scfsi[ch], gr, gr ? &sf[0][ch] : nullptr, &sf[gr][ch]);
                int is[576];
                int status = huffman(br, h, g, p0 + g.part23, is, &nonzero[ch]);
                if (status < 0) return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: invalid Huffman table select");
                ++st->granules;
                if (status == 0) ++st->exact;
                else ++st->overrun;
                if (strict && status != 0)
                    return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: Huffman data overran part2_3_length");
                br.pos = p0 + g.part23;
                requantize(h, g, sf[gr][ch], is, xr[ch]);
            }
            if (h.mode == 1 && h.channels == 2) stereo(h, si.gr[gr], sf[gr][1], xr, nonzero);
            for (int ch = 0; ch < nch_; ++ch) {
                const Granule& g = si.gr[gr][ch];
                double sub[18][32];
                hybrid(h, g, xr[ch], ch, sub);
                synth(ch, sub, pcm[ch]);
            }
        }
        trim_reservoir();
        return 0;
    }

   private:
    int nch_;
    std::vector<uint8_t> res_;
    double overlap_[2][32][18];
    double vbuf_[2][1024];
    int voff_[2];

    void trim_reservoir() {  // main_data_begin reaches back at most 511 bytes
        if (res_.size() > 4096) res_.erase(res_.begin(), res_.end() - 2048);
    }

    // 2.4.1.7 / 2.4.2.7 scale factors, MPEG-1 (scfsi: granule 1 reuses granule 0's groups)
    static void read_sf_mpeg1(BitReader& b, const Granule& g, const int* scfsi, int gr, const ScaleFactors* prev,
                              ScaleFactors* o) {
        std::memset(o, 0, sizeof(*o));
        int s1 = kSlen[0][g.sfc], s2 = kSlen[1][g.sfc];
        if (g.ws && g.block_type == 2) {
            int sfb0 = 0;
            if (g.mixed) {
                for (int sfb = 0; sfb < 8; ++sfb) o->l[sfb] = (int)b.get(s1);
                sfb0 = 3;
            }
            for (int sfb = sfb0; sfb < 12; ++sfb)
                for (int w = 0; w < 3; ++w) o->s[sfb][w] = (int)b.get(sfb < 6 ? s1 : s2);
            return;
        }
        const int bounds[5] = {0, 6, 11, 16, 21};
        for (int grp = 0; grp < 4; ++grp)
            for (int sfb = bounds[grp]; sfb < bounds[grp + 1]; ++sfb) {
                if (gr == 1 && scfsi[grp] && prev) o->l[sfb] = prev->l[sfb];
                else o->l[sfb] = (int)b.get(grp < 2 ? s1 : s2);
            }
    }

    // ISO/IEC 13818-3 2.4.3.2 scale factors of the low sampling frequencies
    static void read_sf_lsf(BitReader& b, const Header& h, Granule& g, int ch, ScaleFactors* o) {
        std::memset(o, 0, sizeof(*o));
        int slen[4] = {0, 0, 0, 0}, tbl;
        int sfc = g.sfc;
        bool is_right = (h.mode_ext & 1) && ch == 1;
        if (!is_right) {
            if (sfc < 400) {
                slen[0] = (sfc >> 4) / 5; slen[1] = (sfc >> 4) % 5; slen[2] = (sfc & 15) >> 2; slen[3] = sfc & 3;
                tbl = 0;
            } else if (sfc < 500) {
                sfc -= 400;
                slen[0] = (sfc >> 2) / 5; slen[1] = (sfc >> 2) % 5; slen[2] = sfc & 3;
                tbl = 1;
            } else {
                sfc -= 500;
                slen[0] = sfc / 3; slen[1] = sfc % 3;
                g.preflag = 1;
                tbl = 2;
            }
        } else {
            int isfc = sfc >> 1;
            if (isfc < 180) {
                slen[0] = isfc / 36; slen[1] = (isfc % 36) / 6; slen[2] = (isfc % 36) % 6;
                tbl = 3;
            } else if (isfc < 244) {
                isfc -= 180;
                slen[0] = (isfc & 63) >> 4; slen[1] = (isfc & 15) >> 2; slen[2] = isfc & 3;
                tbl = 4;
            } else {
                isfc -= 244;
                slen[0] = isfc / 3; slen[1] = isfc % 3;
                tbl = 5;
            }
        }
        int blk = (g.ws && g.block_type == 2) ? (g.mixed ? 2 : 1) : 0;
        int flat[45], fslen[45], n = 0;
        for (int part = 0; part < 4; ++part)
            for (int k = 0; k < kNrSfb[tbl][blk][part]; ++k) {
                flat[n] = (int)b.get(slen[part]);
                fslen[n++] = slen[part];
            }
        int i = 0;
        if (blk == 0) {
            for (int sfb = 0; sfb < 21 && i < n; ++sfb, ++i) { o->l[sfb] = flat[i]; o->lslen[sfb] = fslen[i]; }
        } else {
            int sfb0 = 0;
            if (blk == 2) {
                for (int sfb = 0; sfb < 6; ++sfb, ++i) { o->l[sfb] = flat[i]; o->lslen[sfb] = fslen[i]; }
                sfb0 = 3;
            }
            for (int sfb = sfb0; sfb < 12 && i < n; ++sfb) {
                for (int w = 0; w < 3; ++w, ++i) o->s[sfb][w] = flat[i];
                o->sslen[sfb] = fslen[i - 1];
            }
        }
    }

    // 2.4.2.7 Huffman decoding of big values and count1 quadruples.  Returns 0 when the data ends exactly at
    // part2_3_length, 1 when the last count1 quadruple crossed it (discarded, as every decoder does), -1 on a
    // table select that does not exist.
    static int huffman(BitReader& b, const Header& h, const Granule& g, int64_t end, int* is, int* nonzero) {
        const Tables& T = tabs();
        std::memset(is, 0, 576 * sizeof(int));
        int big = g.big_values * 2;
        int r1, r2;
        if (g.ws) {
            r1 = (g.block_type == 2 || h.sfreq <= 2) ? 36 : h.sfreq != 8 ? 54 : 108;
            r2 = 576;
        } else {
            r1 = kSfbLong[h.sfreq][std::min(g.region0 + 1, 22)];
            r2 = kSfbLong[h.sfreq][std::min(g.region0 + g.region1 + 2, 22)];
        }
        r1 = std::min(r1, big);
        r2 = std::min(r2, big);
        int i = 0;
        for (int region = 0; region < 3; ++region) {
            int stop = region == 0 ? r1 : region == 1 ? r2 : big;
            int tid = g.table[region];
            if (tid == 4 || tid == 14) return -1;
            if (tid == 0) {
                for (; i < stop; ++i) is[i] = 0;
                continue;
            }
            const Tree& tr = T.big[tid < 16 ? tid : tid < 24 ? 16 : 24];
            int n = T.size[tid], lb = T.linbits[tid];
            for (; i < stop; i += 2) {
                int at = 0, leaf;
                for (;;) {
                    int32_t c = tr.node[2 * at + b.bit()];
                    if (c < 0) { leaf = -c - 1; break; }
                    at = c;
                }
                int x = leaf / n, y = leaf % n;
                if (lb && x == 15) x += (int)b.get(lb);
                if (x && b.bit()) x = -x;
                if (lb && y == 15) y += (int)b.get(lb);
                if (y && b.bit()) y = -y;
                is[i] = x;
                is[i + 1] = y;
            }
        }
        int status = 0;
        const Tree& q = T.big[32];
        while (i + 4 <= 576 && b.pos < end) {
            int v;
            if (g.count1_table) {
                v = 15 - (int)b.get(4);
            } else {
                int at = 0;
                for (;;) {
                    int32_t c = q.node[2 * at + b.bit()];
                    if (c < 0) { v = -c - 1; break; }
                    at = c;
                }
            }
            int vals[4] = {(v >> 3) & 1, (v >> 2) & 1, (v >> 1) & 1, v & 1};
            for (int k = 0; k < 4; ++k)
                if (vals[k] && b.bit()) vals[k] = -1;
            if (b.pos > end) {  // the quadruple crossed the end of part2_3: discard it
                status = 1;
                break;
            }
            for (int k = 0; k < 4; ++k) is[i + k] = vals[k];
            i += 4;
        }
        if (b.pos > end && status == 0) status = 1;  // big values already ran past part2_3_length
        int last = 0;
        for (int k = 0; k < 576; ++k)
            if (is[k]) last = k + 1;
        *nonzero = last;
        return status;
    }

    // 2.4.3.4.7 requantisation; short-block lines are left in the transmitted order (band, window, line)
    static void requantize(const Header& h, const Granule& g, const ScaleFactors& sf, const int* is, double* xr) {
        const Tables& T = tabs();
        double gain = std::pow(2.0, 0.25 * (g.global_gain - 210));
        double mul = 0.5 * (1 + g.sf_scale);
        auto val = [&](int q) { return q >= 0 ? T.pow43[q] : -T.pow43[-q]; };
        const int* L = kSfbLong[h.sfreq];
        const int* S = kSfbShort[h.sfreq];
        bool short_blk = g.ws && g.block_type == 2;
        int long_end = !short_blk ? 576 : g.mixed ? (h.lsf ? L[6] : L[8]) : 0;
        for (int sfb = 0; sfb < 22 && L[sfb] < long_end; ++sfb) {
            double f = gain * std::pow(2.0, -mul * (sf.l[sfb] + (g.preflag ? kPretab[sfb] : 0)));
            for (int k = L[sfb]; k < L[sfb + 1] && k < long_end; ++k) xr[k] = is[k] ? val(is[k]) * f : 0.0;
        }
        if (!short_blk) return;
        for (int sfb = g.mixed ? 3 : 0; sfb < 13; ++sfb) {
            int w0 = S[sfb], width = S[sfb + 1] - S[sfb];
            for (int w = 0; w < 3; ++w) {
                double f = gain * std::pow(2.0, -2.0 * g.subblock_gain[w]) * std::pow(2.0, -mul * sf.s[sfb][w]);
                for (int k = 0; k < width; ++k) {
                    int at = 3 * w0 + w * width + k;
                    xr[at] = is[at] ? val(is[at]) * f : 0.0;
                }
            }
        }
    }

    // 2.4.3.4.9 joint stereo: mid/side and intensity (MPEG-1 ratios tan(is_pos pi / 12); MPEG-2 powers of
    // 2^(-1/4) or 2^(-1/2) by intensity_scale)
    static void stereo(const Header& h, const Granule* g, const ScaleFactors& sfr, double xr[2][576], const int* nz) {
        bool ms = h.mode_ext & 2, inten = h.mode_ext & 1;
        const Granule& gr = g[1];
        const int* L = kSfbLong[h.sfreq];
        const int* S = kSfbShort[h.sfreq];
        const double r2 = 1.0 / std::sqrt(2.0);
        bool is_line[576];
        std::memset(is_line, 0, sizeof(is_line));
        double kl[576], kr[576];
        if (inten) {
            const double pi = 3.14159265358979323846;
            auto ratio = [&](int pos, int slen, double* a, double* bb) -> bool {
                if (!h.lsf) {
                    if (pos >= 7) return false;
                    double t = std::tan(pos * pi / 12);
                    *a = t / (1 + t);
                    *bb = 1 / (1 + t);
                    return true;
                }
                if (pos == (1 << slen) - 1) return false;  // illegal intensity position
                double io = (gr.sfc & 1) ? r2 : std::pow(2.0, -0.25);
                if (pos == 0) { *a = 1; *bb = 1; }
                else if (pos & 1) { *a = std::pow(io, (pos + 1) / 2); *bb = 1; }
                else { *a = 1; *bb = std::pow(io, pos / 2); }
                return true;
            };
            bool short_blk = gr.ws && gr.block_type == 2;
            if (!short_blk) {
                int sfb_start = 0;  // first band entirely above the right channel's last nonzero line
                while (sfb_start < 22 && L[sfb_start] < nz[1]) ++sfb_start;
                for (int sfb = sfb_start; sfb < 22; ++sfb) {
                    int src = sfb < 21 ? sfb : 20;
                    double a, bb;
                    if (!ratio(sfr.l[src], sfr.lslen[src], &a, &bb)) continue;
                    for (int k = L[sfb]; k < L[sfb + 1]; ++k) { is_line[k] = true; kl[k] = a; kr[k] = bb; }
                }
            } else {
                for (int w = 0; w < 3; ++w) {
                    int last_sfb = -1;  // last short band of window w holding a nonzero right-channel line
                    for (int sfb = gr.mixed ? 3 : 0; sfb < 13; ++sfb) {
                        int width = S[sfb + 1] - S[sfb];
                        for (int k = 0; k < width; ++k)
                            if (xr[1][3 * S[sfb] + w * width + k] != 0.0) last_sfb = sfb;
                    }
                    int first = std::max(last_sfb + 1, gr.mixed ? 3 : 0);
                    for (int sfb = first; sfb < 13; ++sfb) {
                        int src = sfb < 12 ? sfb : 11;
                        double a, bb;
                        if (!ratio(sfr.s[src][w], sfr.sslen[src], &a, &bb)) continue;
                        int width = S[sfb + 1] - S[sfb];
                        for (int k = 0; k < width; ++k) {
                            int at = 3 * S[sfb] + w * width + k;
                            is_line[at] = true; kl[at] = a; kr[at] = bb;
                        }
                    }
                }
            }
        }
        for (int k = 0; k < 576; ++k) {
            double m = xr[0][k], s = xr[1][k];
            if (is_line[k]) {
                xr[0][k] = m * kl[k];
                xr[1][k] = m * kr[k];
            } else if (ms) {
                xr[0][k] = (m + s) * r2;
                xr[1][k] = (m - s) * r2;
            }
        }
    }

    // 2.4.3.4.10 reorder, antialias, IMDCT with block windows, overlap-add, frequency inversion
    void hybrid(const Header& h, const Granule& g, const double* xr, int ch, double out[18][32]) {
        const Tables& T = tabs();
        bool short_blk = g.ws && g.block_type == 2;
        int long_sb = !short_blk ? 32 : g.mixed ? 2 : 0;
        double lines[576];
        std::memcpy(lines, xr, sizeof(lines));
        // antialias butterflies across the subband boundaries of the long-block part
        for (int sb = 1; sb < long_sb; ++sb)
            for (int i = 0; i < 8; ++i) {
                double a = lines[18 * sb - 1 - i], b = lines[18 * sb + i];
                lines[18 * sb - 1 - i] = a * T.cs[i] - b * T.ca[i];
                lines[18 * sb + i] = b * T.cs[i] + a * T.ca[i];
            }
        // short part: window spectra ws[w][j], j = line index within window w (reorder of 2.4.3.4.8)
        double wsp[3][192];
        if (short_blk) {
            std::memset(wsp, 0, sizeof(wsp));
            const int* S = kSfbShort[h.sfreq];
            for (int sfb = g.mixed ? 3 : 0; sfb < 13; ++sfb) {
                int width = S[sfb + 1] - S[sfb];
                for (int w = 0; w < 3; ++w)
                    for (int k = 0; k < width; ++k) wsp[w][S[sfb] + k] = xr[3 * S[sfb] + w * width + k];
            }
        }
        for (int sb = 0; sb < 32; ++sb) {
            double z[36];
            if (sb < long_sb) {
                int bt = (g.ws && g.mixed && sb < 2) ? 0 : (g.ws ? g.block_type : 0);
                const double* X = lines + 18 * sb;
                for (int i = 0; i < 36; ++i) {
                    double acc = 0;
                    for (int k = 0; k < 18; ++k) acc += X[k] * T.imdct36[i][k];
                    z[i] = acc * T.win[bt][i];
                }
            } else {
                std::memset(z, 0, sizeof(z));
                for (int w = 0; w < 3; ++w) {
                    const double* X = wsp[w] + 6 * sb;
                    for (int i = 0; i < 12; ++i) {
                        double acc = 0;
                        for (int k = 0; k < 6; ++k) acc += X[k] * T.imdct12[i][k];
                        z[6 * w + 6 + i] += acc * T.win12[i];
                    }
                }
            }
            for (int i = 0; i < 18; ++i) {
                double v = z[i] + overlap_[ch][sb][i];
                overlap_[ch][sb][i] = z[18 + i];
                out[i][sb] = (sb & 1) && (i & 1) ? -v : v;  // frequency inversion
            }
        }
    }

    // 2.4.3.4.10.5 polyphase synthesis: V = N S (64 x 32 matrixing), U from V, W = U D, 32 outputs per slot
    void synth(int ch, const double sub[18][32], std::vector<float>& pcm) {
        const Tables& T = tabs();
        double* V = vbuf_[ch];
        for (int t = 0; t < 18; ++t) {
            voff_[ch] = (voff_[ch] - 64) & 1023;
            int o = voff_[ch];
            for (int i = 0; i < 64; ++i) {
                double acc = 0;
                for (int k = 0; k < 32; ++k) acc += T.N[i][k] * sub[t][k];
                V[(o + i) & 1023] = acc;
            }
            for (int j = 0; j < 32; ++j) {
                double acc = 0;
                for (int i = 0; i < 8; ++i) {
                    acc += T.D[64 * i + j] * V[(o + 128 * i + j) & 1023];
                    acc += T.D[64 * i + 32 + j] * V[(o + 128 * i + 96 + j) & 1023];
                }
                pcm.push_back((float)acc);
            }
        }
    }
};

// ---------------------------------------------------------------------------------------------
// Stream walk: ID3v2 skip, frame sync, the Xing / Info frame and its encoder tag
// ---------------------------------------------------------------------------------------------
struct Stream {
    int channels = 0, rate = 0, lsf = 0;
    std::vector<int64_t> frames;  // offsets of the audio frames (the Xing / Info frame excluded)
    int64_t skip = 0;             // leading decoded samples dropped (enc_delay + 529 with an encoder tag)
    // FFmpeg's end discard window [first_discard, last_discard) in decoded sample positions (0 = none)
    int64_t first_discard = 0, last_discard = 0;
    int spf() const { return lsf ? 576 : 1152; }
    // samples of frame k that survive the end discard (the demuxer trims each packet that overlaps the window)
    int64_t frame_keep(int64_t k) const {
        const int64_t n = spf(), s0 = k * n, e0 = s0 + n;
        if (last_discard > 0 && e0 >= first_discard && s0 < last_discard) return n - std::min<int64_t>(e0 - first_discard, n);
        return n;
    }
};

int scan(const uint8_t* buf, int64_t len, Stream* s) {
    int64_t o = 0;
    if (len >= 10 && buf[0] == 'I' && buf[1] == 'D' && buf[2] == '3') {
        int64_t sz = ((int64_t)(buf[6] & 0x7f) << 21) | ((buf[7] & 0x7f) << 14) | ((buf[8] & 0x7f) << 7) |
                     (buf[9] & 0x7f);
        o = 10 + sz + ((buf[5] & 0x10) ? 10 : 0);
    }
    Header first{};
    bool have_first = false, tagged = false;
    int64_t enc_delay = 0, enc_pad = 0, xing_frames = 0;
    while (o + 4 <= len) {
        Header h;
        if (!parse_header(buf + o, &h) || (have_first && (h.sfreq != first.sfreq || h.channels != first.channels))) {
            if (have_first && o + 4 <= len && std::memcmp(buf + o, "TAG", 3) == 0) break;  // ID3v1
            ++o;  // resynchronise
            continue;
        }
        if (!have_first) {
            // a sync word in junk data: require the next frame to start where this one ends (unless at EOF)
            Header h2;
            if (o + h.frame_bytes + 4 <= len && !parse_header(buf + o + h.frame_bytes, &h2)) { ++o; continue; }
        }
        if (o + h.frame_bytes > len) break;  // truncated last frame
        if (!have_first) {
            have_first = true;
            first = h;
            int64_t x = o + 4 + 2 * h.crc + h.side_bytes;
            if (x + 8 <= len && (std::memcmp(buf + x, "Xing", 4) == 0 || std::memcmp(buf + x, "Info", 4) == 0)) {
                uint32_t flags = ((uint32_t)buf[x + 4] << 24) | (buf[x + 5] << 16) | (buf[x + 6] << 8) | buf[x + 7];
                if ((flags & 1) && x + 12 <= len)
                    xing_frames = ((int64_t)buf[x + 8] << 24) | (buf[x + 9] << 16) | (buf[x + 10] << 8) | buf[x + 11];
                int64_t t = x + 8 + ((flags & 1) ? 4 : 0) + ((flags & 2) ? 4 : 0) + ((flags & 4) ? 100 : 0) +
                            ((flags & 8) ? 4 : 0);
                if (t + 24 <= o + h.frame_bytes &&
                    (!std::memcmp(buf + t, "LAME", 4) || !std::memcmp(buf + t, "Lavf", 4) ||
                     !std::memcmp(buf + t, "Lavc", 4))) {
                    uint32_t v = ((uint32_t)buf[t + 21] << 16) | (buf[t + 22] << 8) | buf[t + 23];
                    enc_delay = v >> 12;
                    enc_pad = v & 4095;
                    tagged = true;
                }
                o += h.frame_bytes;  // the tag frame carries no audio
                continue;
            }
            if (x + 4 <= len && o + 36 + 4 <= len && std::memcmp(buf + o + 36, "VBRI", 4) == 0) {
                o += h.frame_bytes;
                continue;
            }
        }
        s->frames.push_back(o);
        o += h.frame_bytes;
    }
    if (!have_first) return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: no MPEG audio Layer III frame found");
    s->channels = first.channels;
    s->rate = kRate[first.sfreq];
    s->lsf = first.lsf;
    if (tagged) {
        s->skip = enc_delay + 529;
        if (xing_frames > 0) {
            s->first_discard = xing_frames * s->spf() - enc_pad + 529;
            s->last_discard = xing_frames * s->spf();
        }
    }
    return 0;
}

int64_t output_samples(const Stream& s) {
    int64_t n = -s.skip;
    for (int64_t k = 0; k < (int64_t)s.frames.size(); ++k) n += s.frame_keep(k);
    return n > 0 ? n : 0;
}

}  // namespace

extern "C" {

int32_t suta_mp3_info(const uint8_t* buf, int64_t len, int32_t* sample_rate, int32_t* channels,
                      int64_t* total_samples) {
    if (!tabs().ok) return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: Huffman tables are not prefix codes");
    Stream s;
    int rc = scan(buf, len, &s);
    if (rc) return rc;
    if (sample_rate) *sample_rate = s.rate;
    if (channels) *channels = s.channels;
    if (total_samples) *total_samples = output_samples(s);
    return SUTA_AUDIO_OK;
}

int32_t suta_mp3_decode(const uint8_t* buf, int64_t len, float* out, int64_t out_capacity, int32_t strict,
                        int64_t* n_out, int64_t* stats) {
    if (!tabs().ok) return fail(SUTA_AUDIO_ERR_FORMAT, "mp3: Huffman tables are not prefix codes");
    Stream s;
    int rc = scan(buf, len, &s);
    if (rc) return rc;
    int64_t total = output_samples(s);
    if (n_out) *n_out = total;
    if (out_capacity < total) return fail(SUTA_AUDIO_ERR_SPACE, "mp3: out_capacity below the decoded length");
    Decoder dec(s.channels);
    std::vector<float> pcm[2];
    Stats st;
    for (int64_t off : s.frames) {
        Header h;
        parse_header(buf + off, &h);
        rc = dec.frame(buf + off, h, pcm, &st, strict != 0);
        if (rc) return rc;
    }
    // kept decoded positions: frame k contributes its first frame_keep(k) samples (from k * spf); the first s.skip
    // kept positions are dropped.  Copied frame by frame with the skip as a running offset (no per-sample index).
    for (int ch = 0; ch < s.channels; ++ch) {
        const int64_t have = (int64_t)pcm[ch].size();
        int64_t pos = -s.skip;  // output index of the frame's first kept sample
        for (int64_t k = 0; k < (int64_t)s.frames.size() && pos < total; ++k) {
            const int64_t n = s.frame_keep(k), base = k * s.spf();
            for (int64_t i = std::max<int64_t>(0, -pos); i < n && pos + i < total; ++i) {
                const int64_t j = base + i;
                out[ch * out_capacity + pos + i] = j < have ? pcm[ch][j] : 0.0f;
            }
            pos += n;
        }
    }
    if (stats) {
        stats[0] = st.frames; stats[1] = st.granules; stats[2] = st.exact; stats[3] = st.overrun; stats[4] = st.lost;
    }
    return SUTA_AUDIO_OK;
}

}  // extern "C"
