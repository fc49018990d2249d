// TFRecord framing writer/reader, used for TensorBoard event files
// (`events.out.tfevents.<ts>.<host>`). In the reference these are
// written by MonitoredTrainingSession's chief-only SummarySaverHook for the
// `loss_<task>` / `accuracy_<task>` scalars (/root/reference/distribute_training.py:128-132,209).
//
// Record = uint64 length | uint32 masked_crc32c(length bytes) | data | uint32 masked_crc32c(data).
#include <cstdio>
#include <memory>
#include <mutex>

#include "common.h"

namespace {

struct RecordWriter {
  FILE* f = nullptr;
  std::mutex mu;
};

struct RecordReader {
  FILE* f = nullptr;
  std::string buf;
};

}  // namespace

TTD_EXPORT void* ttd_record_writer_open(const char* path, int append) {
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  if (!f) {
    ttd::set_error(std::string("cannot open ") + path);
    return nullptr;
  }
  auto* w = new RecordWriter;
  w->f = f;
  return w;
}

TTD_EXPORT int ttd_record_writer_write(void* h, const void* data, uint64_t n) {
  auto* w = static_cast<RecordWriter*>(h);
  std::string hdr;
  ttd::put_fixed64(&hdr, n);
  uint32_t lcrc = ttd::crc32c_mask(ttd::crc32c_value(hdr.data(), 8));
  ttd::put_fixed32(&hdr, lcrc);
  std::string ftr;
  ttd::put_fixed32(&ftr, ttd::crc32c_mask(ttd::crc32c_value(data, n)));
  std::lock_guard<std::mutex> lk(w->mu);
  if (std::fwrite(hdr.data(), 1, hdr.size(), w->f) != hdr.size() ||
      (n && std::fwrite(data, 1, n, w->f) != n) || std::fwrite(ftr.data(), 1, 4, w->f) != 4) {
    ttd::set_error("record write failed");
    return -1;
  }
  return 0;
}

TTD_EXPORT int ttd_record_writer_flush(void* h) {
  auto* w = static_cast<RecordWriter*>(h);
  std::lock_guard<std::mutex> lk(w->mu);
  return std::fflush(w->f);
}

TTD_EXPORT void ttd_record_writer_close(void* h) {
  auto* w = static_cast<RecordWriter*>(h);
  if (!w) return;
  std::fclose(w->f);
  delete w;
}

TTD_EXPORT void* ttd_record_reader_open(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    ttd::set_error(std::string("cannot open ") + path);
    return nullptr;
  }
  auto* r = new RecordReader;
  r->f = f;
  return r;
}

// Reads the next record. Returns its length (>=0), -1 at clean EOF, -2 on corruption.
// The payload stays valid until the next call; fetch it with ttd_record_reader_data.
TTD_EXPORT int64_t ttd_record_reader_next(void* h) {
  auto* r = static_cast<RecordReader*>(h);
  char hdr[12];
  size_t got = std::fread(hdr, 1, 12, r->f);
  if (got == 0) return -1;
  if (got != 12) {
    ttd::set_error("truncated record header");
    return -2;
  }
  uint64_t n = ttd::get_fixed64(hdr);
  if (ttd::crc32c_mask(ttd::crc32c_value(hdr, 8)) != ttd::get_fixed32(hdr + 8)) {
    ttd::set_error("record length crc mismatch");
    return -2;
  }
  r->buf.resize(n);
  char ftr[4];
  if ((n && std::fread(&r->buf[0], 1, n, r->f) != n) || std::fread(ftr, 1, 4, r->f) != 4) {
    ttd::set_error("truncated record payload");
    return -2;
  }
  if (ttd::crc32c_mask(ttd::crc32c_value(r->buf.data(), n)) != ttd::get_fixed32(ftr)) {
    ttd::set_error("record data crc mismatch");
    return -2;
  }
  return static_cast<int64_t>(n);
}

TTD_EXPORT const void* ttd_record_reader_data(void* h) {
  return static_cast<RecordReader*>(h)->buf.data();
}

TTD_EXPORT void ttd_record_reader_close(void* h) {
  auto* r = static_cast<RecordReader*>(h);
  if (!r) return;
  std::fclose(r->f);
  delete r;
}
