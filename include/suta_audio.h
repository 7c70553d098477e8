/*
 * suta_audio.h — C ABI of libsuta_audio.so, the host-side audio decoder of the input pipeline
 * (SURVEY.md section 8f, row f2).
 *
 * The reference reads every utterance with `torchaudio.load(filepath)` (reference data.py:15) and
 * LibriSpeech test-other is FLAC (reference corpus/librispeech.py:30 globs "*.flac").  torchaudio is
 * not installed in this image, so FLAC is decoded here from the format specification (RFC 9639):
 * STREAMINFO, CONSTANT / VERBATIM / FIXED (orders 0-4) / LPC (orders 1-32) subframes, wasted bits,
 * Rice and Rice2 residual partitions with escape codes, the four channel assignments (independent,
 * left/side, side/right, mid/side), fixed and variable blocking, CRC-8 frame-header and CRC-16 frame
 * checks.  Output is what torchaudio.load returns: float32, channel-major (C, N), every sample divided
 * by 2^(bits_per_sample - 1) (exact: a power-of-two scale of an integer of <= 24 significant bits).
 *
 * Entry points (both replace torchaudio.load at reference data.py:15 for .flac files):
 *   suta_flac_info     header only: sample rate, channels, bits per sample, total samples per channel
 *                      (STREAMINFO; 0 = unknown) — the driver's LPT cost model uses it
 *   suta_flac_decode   decode a whole in-memory file
 *
 * MPEG-1 / 2 / 2.5 audio Layer III (CommonVoice clips/<name>.mp3, reference corpus/commonvoice.py:32-38 via
 * torchaudio.load at reference data.py:15), decoded from ISO/IEC 11172-3 / 13818-3 (csrc/mp3.cpp): bit
 * reservoir, MPEG-1 and LSF scale factors, all Huffman tables, long / short / mixed blocks, mid/side and
 * intensity stereo, IMDCT and polyphase synthesis in double precision.  torchaudio's MP3 backend is FFmpeg, so
 * the output follows FFmpeg: float32 in the decoder's native scale, the Xing / Info frame not decoded, and with an
 * encoder tag (LAME / Lavf / Lavc) the first enc_delay + 529 and the last max(0, enc_padding - 529) samples
 * dropped (gapless).  Free-format streams and Layers I / II are refused (SUTA_AUDIO_ERR_FORMAT).
 *   suta_mp3_info      header walk only: sample rate, channels, samples per channel after trimming
 *   suta_mp3_decode    decode a whole in-memory file
 *
 * Conventions: plain pointers and sizes, int32 status codes (0 = OK), a thread-local message via
 * suta_audio_last_error().  Thread-safe: no global state besides the per-thread message, so a loader
 * may decode several files concurrently (ctypes releases the GIL during the call).
 */
#ifndef SUTA_AUDIO_H
#define SUTA_AUDIO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SUTA_AUDIO_OK 0
#define SUTA_AUDIO_ERR_FORMAT 1   /* not a FLAC stream / reserved or invalid field            */
#define SUTA_AUDIO_ERR_CRC 2      /* frame-header CRC-8 or frame CRC-16 mismatch               */
#define SUTA_AUDIO_ERR_TRUNC 3    /* stream ends inside a frame                                */
#define SUTA_AUDIO_ERR_SPACE 4    /* out_capacity too small (required size in *n_out)         */

/* STREAMINFO of the FLAC file held in buf[0..len). */
int32_t suta_flac_info(const uint8_t* buf, int64_t len, int32_t* sample_rate, int32_t* channels,
                       int32_t* bits_per_sample, int64_t* total_samples);

/* Decode every frame.  out: float32 (channels x out_capacity) channel-major buffer; sample i of
 * channel c lands at out[c * out_capacity + i].  *n_out receives the samples per channel decoded.
 * When STREAMINFO states the total, out_capacity must be >= it (else SUTA_AUDIO_ERR_SPACE with the
 * requirement in *n_out).  verify_crc != 0 checks every frame's CRC-8 and CRC-16. */
int32_t suta_flac_decode(const uint8_t* buf, int64_t len, float* out, int64_t out_capacity,
                         int32_t verify_crc, int64_t* n_out);

/* Frame walk of the MP3 file in buf[0..len): sample rate, channels and the samples per channel that
 * suta_mp3_decode will return. */
int32_t suta_mp3_info(const uint8_t* buf, int64_t len, int32_t* sample_rate, int32_t* channels,
                      int64_t* total_samples);

/* Decode every frame into out (float32, channels x out_capacity, channel-major as suta_flac_decode).
 * strict != 0: SUTA_AUDIO_ERR_FORMAT when a granule's Huffman data runs past its part2_3_length (a damaged or
 * mis-parsed stream; decoders otherwise drop the crossing count1 quadruple).  stats (may be NULL) receives
 * 5 int64: frames decoded, granule-channels, of those ending exactly at part2_3_length, overrunning it, and
 * frames whose bit reservoir was not available (decoded as silence). */
int32_t suta_mp3_decode(const uint8_t* buf, int64_t len, float* out, int64_t out_capacity, int32_t strict,
                        int64_t* n_out, int64_t* stats);

const char* suta_audio_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SUTA_AUDIO_H */
