#include "annexb.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "bitstream.h"
#include "h264_syntax.h"

namespace mivc {

namespace {

struct Au {
  size_t start = 0, end = 0;  // byte range in the stream
  bool idr = false;
  bool has_ps = false;        // carries SPS and PPS
};

// first_mb_in_slice of a slice NAL: parse the first ue(v) of the (escaped) payload
int first_mb_of(const uint8_t* p, size_t n) {
  // payload after the header byte; emulation prevention cannot occur in the first bytes of a ue
  // with fewer than 16 leading zeros, so read raw.
  if (n < 2) return -1;
  BitReader br(p + 1, std::min<size_t>(n - 1, 8));
  try {
    return br.get_ue_max((1u << 20) - 1, "first_mb_in_slice");
  } catch (...) {
    return -1;
  }
}

std::vector<Au> access_units(const uint8_t* p, size_t n, const std::vector<NalUnit>& nals) {
  std::vector<Au> aus;
  size_t pending = SIZE_MAX;
  bool pending_sps = false, pending_pps = false;
  for (size_t i = 0; i < nals.size(); ++i) {
    const NalUnit& u = nals[i];
    int t = u.nal_unit_type;
    bool vcl = t >= 1 && t <= 5;
    if (!vcl) {
      if (t == 9 && pending != SIZE_MAX) {
        // an AUD always starts a new access unit
      }
      if (pending == SIZE_MAX || t == 9) pending = u.offset;
      if (t == 7) pending_sps = true;
      if (t == 8) pending_pps = true;
      continue;
    }
    int fm = first_mb_of(p + u.offset + (p[u.offset + 2] == 1 ? 3 : 4), u.size - (p[u.offset + 2] == 1 ? 3 : 4));
    if (fm == 0 || aus.empty()) {
      Au a;
      a.start = pending != SIZE_MAX ? pending : u.offset;
      a.idr = t == 5;
      a.has_ps = pending_sps && pending_pps;
      if (!aus.empty()) aus.back().end = a.start;
      aus.push_back(a);
    } else if (t == 5) {
      aus.back().idr = true;
    }
    pending = SIZE_MAX;
    pending_sps = pending_pps = false;
  }
  if (!aus.empty()) aus.back().end = n;
  return aus;
}

void put32(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back(v >> 24);
  b.push_back(v >> 16);
  b.push_back(v >> 8);
  b.push_back(v);
}
void put16(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back(v >> 8);
  b.push_back(v);
}
void put_str(std::vector<uint8_t>& b, const char* s) { b.insert(b.end(), s, s + std::strlen(s)); }
// box helpers: returns index of size field
size_t begin_box(std::vector<uint8_t>& b, const char* type) {
  size_t at = b.size();
  put32(b, 0);
  put_str(b, type);
  return at;
}
void end_box(std::vector<uint8_t>& b, size_t at) {
  uint32_t sz = static_cast<uint32_t>(b.size() - at);
  b[at] = sz >> 24;
  b[at + 1] = sz >> 16;
  b[at + 2] = sz >> 8;
  b[at + 3] = sz;
}
void full_box_header(std::vector<uint8_t>& b, int version, uint32_t flags) { put32(b, (version << 24) | flags); }
void put_matrix(std::vector<uint8_t>& b) {
  const uint32_t m[9] = {0x00010000, 0, 0, 0, 0x00010000, 0, 0, 0, 0x40000000};
  for (uint32_t v : m) put32(b, v);
}

uint32_t rd32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
uint16_t rd16(const uint8_t* p) { return static_cast<uint16_t>((p[0] << 8) | p[1]); }

}  // namespace

StreamInfo probe_annexb(const uint8_t* p, size_t n) {
  StreamInfo si;
  std::vector<NalUnit> nals = parse_annexb(p, n, true);
  for (const NalUnit& u : nals) {
    if (u.nal_unit_type == 7 && si.width == 0) {
      BitReader br(u.rbsp.data(), u.rbsp.size());
      h264::SPS s = h264::parse_sps(br);
      si.width = s.width_mbs * 16 - 2 * (s.crop_left + s.crop_right);
      si.height = s.height_mbs * 16 - 2 * (s.crop_top + s.crop_bottom);
      si.profile_idc = s.profile_idc;
      si.level_idc = s.level_idc;
      if (s.vui_present && s.num_units_in_tick) si.fps = s.time_scale / (2.0 * s.num_units_in_tick);
    } else if (u.nal_unit_type == 8) {
      BitReader br(u.rbsp.data(), u.rbsp.size());
      br.get_ue();
      br.get_ue();
      si.cabac = br.get_bit();
    }
  }
  std::vector<NalUnit> raw = parse_annexb(p, n, false);
  for (const Au& a : access_units(p, n, raw)) {
    ++si.frames;
    if (a.idr) ++si.idr_frames;
  }
  return si;
}

std::vector<std::pair<size_t, size_t>> split_annexb_at_idr(const uint8_t* p, size_t n, int min_frames) {
  std::vector<NalUnit> raw = parse_annexb(p, n, false);
  std::vector<Au> aus = access_units(p, n, raw);
  std::vector<std::pair<size_t, size_t>> cuts;
  int in_piece = 0;
  for (size_t i = 0; i < aus.size(); ++i) {
    bool cut = cuts.empty() || (aus[i].idr && in_piece >= min_frames);
    if (cut) {
      if (!cuts.empty()) cuts.back().second = aus[i].start - cuts.back().first;
      cuts.emplace_back(aus[i].start, 0);
      in_piece = 0;
    }
    ++in_piece;
  }
  if (!cuts.empty()) cuts.back().second = n - cuts.back().first;
  return cuts;
}

std::vector<std::vector<uint8_t>> split_annexb_pieces(const uint8_t* p, size_t n, int min_frames) {
  std::vector<NalUnit> raw = parse_annexb(p, n, false);
  std::vector<Au> aus = access_units(p, n, raw);
  std::vector<std::vector<uint8_t>> pieces;
  std::vector<uint8_t> last_ps;  // most recent SPS+PPS NAL bytes
  int in_piece = 0;
  size_t ni = 0;
  for (size_t i = 0; i < aus.size(); ++i) {
    // collect parameter sets inside this AU
    std::vector<uint8_t> ps_here;
    while (ni < raw.size() && raw[ni].offset < aus[i].end) {
      if (raw[ni].nal_unit_type == 7 || raw[ni].nal_unit_type == 8)
        ps_here.insert(ps_here.end(), p + raw[ni].offset, p + raw[ni].offset + raw[ni].size);
      ++ni;
    }
    bool cut = pieces.empty() || (aus[i].idr && in_piece >= min_frames);
    if (cut) {
      pieces.emplace_back();
      if (!aus[i].has_ps && !last_ps.empty()) pieces.back() = last_ps;
      in_piece = 0;
    }
    if (!ps_here.empty()) last_ps = ps_here;
    pieces.back().insert(pieces.back().end(), p + aus[i].start, p + aus[i].end);
    ++in_piece;
  }
  return pieces;
}

std::vector<uint8_t> concat_annexb(const std::vector<std::pair<const uint8_t*, size_t>>& parts) {
  std::vector<uint8_t> out;
  size_t total = 0;
  for (auto& pr : parts) total += pr.second;
  out.reserve(total);
  for (auto& pr : parts) {
    if (pr.second < 4) continue;
    // every piece must start with a start code
    bool sc = (pr.first[0] == 0 && pr.first[1] == 0 && (pr.first[2] == 1 || (pr.first[2] == 0 && pr.first[3] == 1)));
    if (!sc) throw std::runtime_error("concat: piece does not start with an Annex-B start code");
    out.insert(out.end(), pr.first, pr.first + pr.second);
  }
  return out;
}

std::vector<uint8_t> mux_mp4(const uint8_t* p, size_t n, double fps) {
  std::vector<NalUnit> raw = parse_annexb(p, n, false);
  std::vector<NalUnit> esc = parse_annexb(p, n, true);
  std::vector<Au> aus = access_units(p, n, raw);
  if (aus.empty()) throw std::runtime_error("mp4 mux: no access units");
  // parameter sets (first of each)
  std::vector<uint8_t> sps, pps;
  int width = 0, height = 0;
  for (size_t i = 0; i < raw.size(); ++i) {
    size_t hdr = raw[i].offset + (p[raw[i].offset + 2] == 1 ? 3 : 4);
    size_t len = raw[i].offset + raw[i].size - hdr;
    while (len > 0 && p[hdr + len - 1] == 0) --len;
    if (raw[i].nal_unit_type == 7 && sps.empty()) {
      sps.assign(p + hdr, p + hdr + len);
      BitReader br(esc[i].rbsp.data(), esc[i].rbsp.size());
      h264::SPS s = h264::parse_sps(br);
      width = s.width_mbs * 16 - 2 * (s.crop_left + s.crop_right);
      height = s.height_mbs * 16 - 2 * (s.crop_top + s.crop_bottom);
      if (fps <= 0 && s.vui_present && s.num_units_in_tick) fps = s.time_scale / (2.0 * s.num_units_in_tick);
    }
    if (raw[i].nal_unit_type == 8 && pps.empty()) pps.assign(p + hdr, p + hdr + len);
  }
  if (sps.empty() || pps.empty()) throw std::runtime_error("mp4 mux: stream has no SPS/PPS");
  if (fps <= 0) fps = 30.0;
  // samples: AVCC (4-byte length) NALs excluding SPS/PPS/AUD
  std::vector<uint8_t> mdat_payload;
  std::vector<uint32_t> sizes;
  std::vector<uint32_t> sync;
  size_t ni = 0;
  for (size_t a = 0; a < aus.size(); ++a) {
    size_t before = mdat_payload.size();
    while (ni < raw.size() && raw[ni].offset < aus[a].end) {
      int t = raw[ni].nal_unit_type;
      if (t != 7 && t != 8 && t != 9) {
        size_t hdr = raw[ni].offset + (p[raw[ni].offset + 2] == 1 ? 3 : 4);
        size_t len = raw[ni].offset + raw[ni].size - hdr;
        while (len > 0 && p[hdr + len - 1] == 0) --len;
        put32(mdat_payload, static_cast<uint32_t>(len));
        mdat_payload.insert(mdat_payload.end(), p + hdr, p + hdr + len);
      }
      ++ni;
    }
    sizes.push_back(static_cast<uint32_t>(mdat_payload.size() - before));
    if (aus[a].idr) sync.push_back(static_cast<uint32_t>(a + 1));
  }
  uint32_t timescale = static_cast<uint32_t>(fps * 1000.0 + 0.5);
  uint32_t delta = 1000;
  uint32_t nsamples = static_cast<uint32_t>(sizes.size());
  uint32_t media_dur = nsamples * delta;
  uint32_t movie_dur = static_cast<uint32_t>(nsamples * 1000.0 / fps + 0.5);

  std::vector<uint8_t> out;
  size_t b = begin_box(out, "ftyp");
  put_str(out, "isom");
  put32(out, 512);
  put_str(out, "isomiso2avc1mp41");
  end_box(out, b);

  size_t moov = begin_box(out, "moov");
  size_t mvhd = begin_box(out, "mvhd");
  full_box_header(out, 0, 0);
  put32(out, 0);
  put32(out, 0);
  put32(out, 1000);
  put32(out, movie_dur);
  put32(out, 0x00010000);
  put16(out, 0x0100);
  put16(out, 0);
  put32(out, 0);
  put32(out, 0);
  put_matrix(out);
  for (int i = 0; i < 6; ++i) put32(out, 0);
  put32(out, 2);
  end_box(out, mvhd);
  size_t trak = begin_box(out, "trak");
  size_t tkhd = begin_box(out, "tkhd");
  full_box_header(out, 0, 3);
  put32(out, 0);
  put32(out, 0);
  put32(out, 1);
  put32(out, 0);
  put32(out, movie_dur);
  put32(out, 0);
  put32(out, 0);
  put16(out, 0);
  put16(out, 0);
  put16(out, 0);
  put16(out, 0);
  put_matrix(out);
  put32(out, static_cast<uint32_t>(width) << 16);
  put32(out, static_cast<uint32_t>(height) << 16);
  end_box(out, tkhd);
  size_t mdia = begin_box(out, "mdia");
  size_t mdhd = begin_box(out, "mdhd");
  full_box_header(out, 0, 0);
  put32(out, 0);
  put32(out, 0);
  put32(out, timescale);
  put32(out, media_dur);
  put16(out, 0x55C4);  // 'und'
  put16(out, 0);
  end_box(out, mdhd);
  size_t hdlr = begin_box(out, "hdlr");
  full_box_header(out, 0, 0);
  put32(out, 0);
  put_str(out, "vide");
  put32(out, 0);
  put32(out, 0);
  put32(out, 0);
  put_str(out, "VideoHandler");
  out.push_back(0);
  end_box(out, hdlr);
  size_t minf = begin_box(out, "minf");
  size_t vmhd = begin_box(out, "vmhd");
  full_box_header(out, 0, 1);
  put16(out, 0);
  put16(out, 0);
  put16(out, 0);
  put16(out, 0);
  end_box(out, vmhd);
  size_t dinf = begin_box(out, "dinf");
  size_t dref = begin_box(out, "dref");
  full_box_header(out, 0, 0);
  put32(out, 1);
  size_t url = begin_box(out, "url ");
  full_box_header(out, 0, 1);
  end_box(out, url);
  end_box(out, dref);
  end_box(out, dinf);
  size_t stbl = begin_box(out, "stbl");
  size_t stsd = begin_box(out, "stsd");
  full_box_header(out, 0, 0);
  put32(out, 1);
  size_t avc1 = begin_box(out, "avc1");
  for (int i = 0; i < 6; ++i) out.push_back(0);
  put16(out, 1);
  put16(out, 0);
  put16(out, 0);
  put32(out, 0);
  put32(out, 0);
  put32(out, 0);
  put16(out, static_cast<uint32_t>(width));
  put16(out, static_cast<uint32_t>(height));
  put32(out, 0x00480000);
  put32(out, 0x00480000);
  put32(out, 0);
  put16(out, 1);
  for (int i = 0; i < 32; ++i) out.push_back(0);
  put16(out, 0x0018);
  put16(out, 0xFFFF);
  size_t avcc = begin_box(out, "avcC");
  out.push_back(1);
  out.push_back(sps[1]);
  out.push_back(sps[2]);
  out.push_back(sps[3]);
  out.push_back(0xFF);
  out.push_back(0xE1);
  put16(out, static_cast<uint32_t>(sps.size()));
  out.insert(out.end(), sps.begin(), sps.end());
  out.push_back(1);
  put16(out, static_cast<uint32_t>(pps.size()));
  out.insert(out.end(), pps.begin(), pps.end());
  end_box(out, avcc);
  end_box(out, avc1);
  end_box(out, stsd);
  size_t stts = begin_box(out, "stts");
  full_box_header(out, 0, 0);
  put32(out, 1);
  put32(out, nsamples);
  put32(out, delta);
  end_box(out, stts);
  size_t stss = begin_box(out, "stss");
  full_box_header(out, 0, 0);
  put32(out, static_cast<uint32_t>(sync.size()));
  for (uint32_t s : sync) put32(out, s);
  end_box(out, stss);
  size_t stsc = begin_box(out, "stsc");
  full_box_header(out, 0, 0);
  put32(out, 1);
  put32(out, 1);
  put32(out, nsamples);
  put32(out, 1);
  end_box(out, stsc);
  size_t stsz = begin_box(out, "stsz");
  full_box_header(out, 0, 0);
  put32(out, 0);
  put32(out, nsamples);
  for (uint32_t s : sizes) put32(out, s);
  end_box(out, stsz);
  size_t stco = begin_box(out, "stco");
  full_box_header(out, 0, 0);
  put32(out, 1);
  size_t chunk_off_at = out.size();
  put32(out, 0);
  end_box(out, stco);
  end_box(out, stbl);
  end_box(out, minf);
  end_box(out, mdia);
  end_box(out, trak);
  end_box(out, moov);
  // mdat (32-bit size; pieces are far below 4 GiB)
  uint64_t mdat_size = 8 + mdat_payload.size();
  if (mdat_size > 0xFFFFFFFFull) throw std::runtime_error("mp4 mux: mdat too large");
  uint32_t data_off = static_cast<uint32_t>(out.size() + 8);
  out[chunk_off_at] = data_off >> 24;
  out[chunk_off_at + 1] = data_off >> 16;
  out[chunk_off_at + 2] = data_off >> 8;
  out[chunk_off_at + 3] = data_off;
  put32(out, static_cast<uint32_t>(mdat_size));
  put_str(out, "mdat");
  out.insert(out.end(), mdat_payload.begin(), mdat_payload.end());
  return out;
}

H264Samples h264_samples(const uint8_t* p, size_t n) {
  std::vector<NalUnit> raw = parse_annexb(p, n, false);
  std::vector<Au> aus = access_units(p, n, raw);
  if (aus.empty()) throw std::runtime_error("h264_samples: no access units");
  H264Samples out;
  std::vector<h264::SPS> sps_tab(32);
  std::vector<h264::PPS> pps_tab(256);
  std::vector<char> have_sps(32, 0), have_pps(256, 0);
  auto unescape = [&](size_t b, size_t e, size_t cap) {
    std::vector<uint8_t> r;
    r.reserve(std::min(e - b, cap));
    int zeros = 0;
    for (size_t j = b; j < e && r.size() < cap; ++j) {
      uint8_t c = p[j];
      if (zeros >= 2 && c == 3) {
        zeros = 0;
        continue;
      }
      r.push_back(c);
      zeros = (c == 0) ? zeros + 1 : 0;
    }
    return r;
  };
  // POC state (8.2.1): previous reference picture's msb/lsb (type 0), previous picture's
  // frame_num / FrameNumOffset (types 1 and 2)
  int prev_msb = 0, prev_lsb = 0, prev_fn = 0, prev_fno = 0;
  long long epoch = 0;
  bool prev_mmco5 = false;
  std::vector<std::pair<long long, long long>> keys;  // (epoch, poc) per sample
  size_t ni = 0;
  for (size_t a = 0; a < aus.size(); ++a) {
    size_t before = out.data.size();
    bool have_key = false;
    while (ni < raw.size() && raw[ni].offset < aus[a].end) {
      const NalUnit& u = raw[ni++];
      int t = u.nal_unit_type;
      size_t hdr = u.offset + (p[u.offset + 2] == 1 ? 3 : 4);
      size_t len = u.offset + u.size - hdr;
      while (len > 0 && p[hdr + len - 1] == 0) --len;
      if (len == 0) continue;
      if (t == 7 || t == 8) {
        std::vector<uint8_t> rb = unescape(hdr + 1, hdr + len, SIZE_MAX);
        BitReader br(rb.data(), rb.size());
        if (t == 7) {
          h264::SPS s = h264::parse_sps(br);
          if (s.sps_id < 0 || s.sps_id > 31) throw std::runtime_error("h264_samples: bad sps id");
          sps_tab[s.sps_id] = s;
          have_sps[s.sps_id] = 1;
          if (out.sps.empty()) {
            out.sps.assign(p + hdr, p + hdr + len);
            out.width = s.width_mbs * 16 - 2 * (s.crop_left + s.crop_right);
            out.height = s.height_mbs * 16 - 2 * (s.crop_top + s.crop_bottom);
            if (s.vui_present && s.num_units_in_tick) out.fps = s.time_scale / (2.0 * s.num_units_in_tick);
          }
        } else {
          h264::PPS q = h264::parse_pps(br, sps_tab.data());
          if (q.pps_id < 0 || q.pps_id > 255) throw std::runtime_error("h264_samples: bad pps id");
          pps_tab[q.pps_id] = q;
          have_pps[q.pps_id] = 1;
          if (out.pps.empty()) out.pps.assign(p + hdr, p + hdr + len);
        }
        continue;
      }
      if (t != 9) {
        put32(out.data, static_cast<uint32_t>(len));
        out.data.insert(out.data.end(), p + hdr, p + hdr + len);
      }
      if (have_key || t < 1 || t > 5) continue;
      have_key = true;
      // slice headers with long reference-list modifications / weight tables stay within 4 KiB
      std::vector<uint8_t> rb = unescape(hdr + 1, hdr + len, 4096);
      BitReader br(rb.data(), rb.size());
      h264::SliceHeader h = h264::parse_slice_header(br, t, u.nal_ref_idc, sps_tab.data(), pps_tab.data());
      if (!have_pps[h.pps_id] || !have_sps[pps_tab[h.pps_id].sps_id])
        throw std::runtime_error("h264_samples: slice before its parameter sets");
      const h264::SPS& sp = sps_tab[pps_tab[h.pps_id].sps_id];
      bool idr = t == 5;
      if (idr || prev_mmco5) {
        ++epoch;
        prev_msb = prev_lsb = 0;
        prev_fno = 0;
        if (prev_mmco5) prev_fn = 0;
      }
      long long poc = 0;
      int fno = 0;
      int max_fn = 1 << sp.log2_max_frame_num;
      if (sp.poc_type == 0) {
        int max_lsb = 1 << sp.log2_max_poc_lsb, lsb = h.poc_lsb, msb;
        if (lsb < prev_lsb && prev_lsb - lsb >= max_lsb / 2) msb = prev_msb + max_lsb;
        else if (lsb > prev_lsb && lsb - prev_lsb > max_lsb / 2) msb = prev_msb - max_lsb;
        else msb = prev_msb;
        poc = msb + lsb;
        if (u.nal_ref_idc) {
          prev_msb = msb;
          prev_lsb = lsb;
        }
      } else {
        if (idr) fno = 0;
        else if (prev_fn > h.frame_num) fno = prev_fno + max_fn;
        else fno = prev_fno;
        if (sp.poc_type == 2) {
          poc = idr ? 0 : (u.nal_ref_idc == 0 ? 2LL * (fno + h.frame_num) - 1 : 2LL * (fno + h.frame_num));
        } else {
          int nc = static_cast<int>(sp.offset_for_ref_frame.size());
          long long abs_fn = nc ? fno + h.frame_num : 0;
          if (u.nal_ref_idc == 0 && abs_fn > 0) --abs_fn;
          long long exp = 0;
          if (abs_fn > 0) {
            long long delta_cycle = 0;
            for (int v : sp.offset_for_ref_frame) delta_cycle += v;
            long long cycle = (abs_fn - 1) / nc, in_cycle = (abs_fn - 1) % nc;
            exp = cycle * delta_cycle;
            for (long long i = 0; i <= in_cycle; ++i) exp += sp.offset_for_ref_frame[i];
          }
          if (u.nal_ref_idc == 0) exp += sp.offset_for_non_ref_pic;
          poc = exp + h.delta_poc[0];
        }
        prev_fno = fno;
        prev_fn = h.frame_num;
      }
      bool mmco5 = false;
      for (const h264::Mmco& m : h.mmco) mmco5 = mmco5 || m.op == 5;
      prev_mmco5 = mmco5;
      keys.emplace_back(epoch, mmco5 ? (1LL << 40) : poc);  // an mmco5 picture follows its epoch
    }
    if (!have_key) throw std::runtime_error("h264_samples: access unit without a slice");
    out.sizes.push_back(static_cast<uint32_t>(out.data.size() - before));
    out.sync.push_back(aus[a].idr ? 1 : 0);
  }
  if (out.sps.empty() || out.pps.empty()) throw std::runtime_error("h264_samples: stream has no SPS/PPS");
  // display index = rank of (epoch, poc)
  std::vector<int32_t> idx(keys.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = static_cast<int32_t>(i);
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t x, int32_t y) { return keys[x] < keys[y]; });
  out.display.assign(keys.size(), 0);
  for (size_t r = 0; r < idx.size(); ++r) out.display[idx[r]] = static_cast<int32_t>(r);
  return out;
}

namespace {
struct BoxRef {
  const uint8_t* p;
  size_t n;
};
bool find_box(const uint8_t* p, size_t n, const char* type, BoxRef* out) {
  size_t i = 0;
  while (i + 8 <= n) {
    uint64_t sz = rd32(p + i);
    size_t hdr = 8;
    if (sz == 1) {
      if (i + 16 > n) return false;
      sz = (uint64_t(rd32(p + i + 8)) << 32) | rd32(p + i + 12);
      hdr = 16;
    } else if (sz == 0) {
      sz = n - i;
    }
    if (sz < hdr || i + sz > n) return false;
    if (std::memcmp(p + i + 4, type, 4) == 0) {
      out->p = p + i + hdr;
      out->n = static_cast<size_t>(sz - hdr);
      return true;
    }
    i += static_cast<size_t>(sz);
  }
  return false;
}
BoxRef must(const BoxRef& in, const char* type) {
  BoxRef r{};
  if (!find_box(in.p, in.n, type, &r)) throw std::runtime_error(std::string("mp4 demux: missing box ") + type);
  return r;
}
}  // namespace

std::vector<uint8_t> demux_mp4_to_annexb(const uint8_t* p, size_t n) {
  // every read is checked against its box (workers parse network-fetched pieces;
  // tests/test_fuzz_parsers.py runs this under ASan + UBSan)
  auto need = [](const BoxRef& b, size_t off, size_t len, const char* what) {
    if (off > b.n || len > b.n - off) throw std::runtime_error(std::string("mp4 demux: truncated ") + what);
  };
  BoxRef file{p, n};
  BoxRef moov = must(file, "moov");
  BoxRef trak = must(moov, "trak");
  BoxRef mdia = must(trak, "mdia");
  BoxRef minf = must(mdia, "minf");
  BoxRef st = must(minf, "stbl");
  BoxRef stsd = must(st, "stsd");
  // stsd: fullbox(4) entry_count(4) then sample entry box
  need(stsd, 0, 8, "stsd");
  BoxRef entries{stsd.p + 8, stsd.n - 8};
  BoxRef avc1 = must(entries, "avc1");
  need(avc1, 0, 78, "avc1");
  BoxRef avcc_parent{avc1.p + 78, avc1.n - 78};
  BoxRef avcc = must(avcc_parent, "avcC");
  need(avcc, 0, 6, "avcC");
  const uint8_t* c = avcc.p;
  int len_size = (c[4] & 3) + 1;
  std::vector<uint8_t> ps;
  size_t off = 5;
  static const uint8_t sc[4] = {0, 0, 0, 1};
  for (int list = 0; list < 2; ++list) {
    need(avcc, off, 1, "avcC");
    int cnt = list == 0 ? (c[off] & 31) : c[off];
    ++off;
    for (int i = 0; i < cnt; ++i) {
      need(avcc, off, 2, "avcC");
      size_t l = rd16(c + off);
      off += 2;
      need(avcc, off, l, "avcC parameter set");
      ps.insert(ps.end(), sc, sc + 4);
      ps.insert(ps.end(), c + off, c + off + l);
      off += l;
    }
  }
  BoxRef stsz = must(st, "stsz");
  need(stsz, 0, 12, "stsz");
  uint32_t fixed = rd32(stsz.p + 4), count = rd32(stsz.p + 8);
  if (!fixed) need(stsz, 12, size_t(count) * 4, "stsz");
  if (count > n) throw std::runtime_error("mp4 demux: more samples than bytes");
  std::vector<uint32_t> sizes(count);
  for (uint32_t i = 0; i < count; ++i) sizes[i] = fixed ? fixed : rd32(stsz.p + 12 + 4 * i);
  std::vector<uint64_t> chunks;
  BoxRef co{};
  if (find_box(st.p, st.n, "stco", &co)) {
    need(co, 0, 8, "stco");
    uint32_t nc = rd32(co.p + 4);
    need(co, 8, size_t(nc) * 4, "stco");
    for (uint32_t i = 0; i < nc; ++i) chunks.push_back(rd32(co.p + 8 + 4 * i));
  } else {
    co = must(st, "co64");
    need(co, 0, 8, "co64");
    uint32_t nc = rd32(co.p + 4);
    need(co, 8, size_t(nc) * 8, "co64");
    for (uint32_t i = 0; i < nc; ++i) chunks.push_back((uint64_t(rd32(co.p + 8 + 8 * i)) << 32) | rd32(co.p + 12 + 8 * i));
  }
  BoxRef stsc = must(st, "stsc");
  need(stsc, 0, 8, "stsc");
  uint32_t nent = rd32(stsc.p + 4);
  need(stsc, 8, size_t(nent) * 12, "stsc");
  if (nent == 0) throw std::runtime_error("mp4 demux: empty stsc");
  std::vector<uint32_t> first_chunk(nent), per_chunk(nent);
  for (uint32_t i = 0; i < nent; ++i) {
    first_chunk[i] = rd32(stsc.p + 8 + 12 * i);
    per_chunk[i] = rd32(stsc.p + 12 + 12 * i);
  }
  std::vector<uint32_t> syncs;
  BoxRef stss{};
  bool have_stss = find_box(st.p, st.n, "stss", &stss);
  if (have_stss) {
    need(stss, 0, 8, "stss");
    uint32_t ns = rd32(stss.p + 4);
    need(stss, 8, size_t(ns) * 4, "stss");
    for (uint32_t i = 0; i < ns; ++i) syncs.push_back(rd32(stss.p + 8 + 4 * i));
  }
  std::vector<uint8_t> out;
  uint32_t sample = 0;
  size_t si = 0, ei = 0;
  uint32_t spc = per_chunk[0];
  for (size_t ch = 0; ch < chunks.size() && sample < count; ++ch) {
    uint32_t chunk_no = static_cast<uint32_t>(ch + 1);
    while (ei < nent && first_chunk[ei] <= chunk_no) spc = per_chunk[ei++];
    uint64_t pos = chunks[ch];
    for (uint32_t k = 0; k < spc && sample < count; ++k, ++sample) {
      bool is_sync = !have_stss;
      while (si < syncs.size() && syncs[si] < sample + 1) ++si;
      if (si < syncs.size() && syncs[si] == sample + 1) is_sync = true;
      if (is_sync) out.insert(out.end(), ps.begin(), ps.end());
      uint64_t end = pos + sizes[sample];
      if (pos > n || end > n) throw std::runtime_error("mp4 demux: sample outside file");
      uint64_t q = pos;
      while (q + len_size <= end) {
        uint32_t l = 0;
        for (int b = 0; b < len_size; ++b) l = (l << 8) | p[q + b];
        q += len_size;
        if (q + l > end) throw std::runtime_error("mp4 demux: bad NAL length");
        out.insert(out.end(), sc, sc + 4);
        out.insert(out.end(), p + q, p + q + l);
        q += l;
      }
      pos = end;
    }
  }
  return out;
}

}  // namespace mivc
