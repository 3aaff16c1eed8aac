// Compressed-stream segment I/O: probe, keyframe-aligned split, ordered concat,
// and a minimal ISO-BMFF (MP4) mux/demux.
//
// Reference parity:
//   * probe   <- GetSumTime's `ffmpeg -i` + Duration regex (server.go:239-265)
//   * split   <- SplitFile's `ffmpeg -f segment -segment_time T -c copy` (server.go:193-204):
//                cut at the first keyframe at or after each boundary, each piece restarts
//                with parameter sets (the analogue of -reset_timestamps 1)
//   * concat  <- concat.sh `ffmpeg -f concat -i filelist.txt -c copy` (server.go:349-361)
//   * mp4     <- the `.mp4` container every reference piece uses (server.go:200, client.go:54)
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

namespace mivc {

struct StreamInfo {
  int width = 0, height = 0;
  double fps = 0.0;
  int frames = 0;
  int idr_frames = 0;
  int profile_idc = 0, level_idc = 0;
  bool cabac = false;
};

StreamInfo probe_annexb(const uint8_t* p, size_t n);

// Split into pieces that each start at an IDR access unit (including the SPS/PPS
// that precede it; the most recent SPS/PPS are re-emitted if the IDR has none).
// A new piece starts at an IDR only once >= min_frames pictures are in the current one.
// Returns (offset, size) of each piece in the input.  Pieces that need parameter-set
// injection are reported with the same offsets; use split_annexb_pieces for bytes.
std::vector<std::pair<size_t, size_t>> split_annexb_at_idr(const uint8_t* p, size_t n, int min_frames);
std::vector<std::vector<uint8_t>> split_annexb_pieces(const uint8_t* p, size_t n, int min_frames);

// Ordered concatenation of Annex-B pieces.
std::vector<uint8_t> concat_annexb(const std::vector<std::pair<const uint8_t*, size_t>>& parts);

// Annex-B H.264 elementary stream -> MP4 (one video track) and back.
std::vector<uint8_t> mux_mp4(const uint8_t* p, size_t n, double fps);
std::vector<uint8_t> demux_mp4_to_annexb(const uint8_t* p, size_t n);

// MP4 sample view of an H.264 Annex-B stream (for the ISO-BMFF writer in
// govideocompressor_amd/segment/mp4.py): one sample per access unit in decoding order,
// NALs as 4-byte-length AVCC units without SPS/PPS/AUD, sync = IDR, and the display index
// of every sample from its picture order count (8.2.1, POC types 0/1/2; an IDR or a
// memory_management_control_operation 5 starts a new display epoch), which the writer
// turns into composition offsets (ctts) for B pictures.
struct H264Samples {
  std::vector<uint8_t> data;
  std::vector<uint32_t> sizes;
  std::vector<uint8_t> sync;
  std::vector<int32_t> display;
  std::vector<uint8_t> sps, pps;  // first SPS / PPS NAL (header byte + escaped payload)
  int width = 0, height = 0;
  double fps = 0.0;
};
H264Samples h264_samples(const uint8_t* p, size_t n);

}  // namespace mivc
