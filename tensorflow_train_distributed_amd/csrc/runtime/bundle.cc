// TensorBundle V2 checkpoint writer / reader / merger (the on-disk format of TF's
// Saver V2 and tf.train.Checkpoint).
//
// The reference never calls the Saver directly: MonitoredTrainingSession(checkpoint_dir=...,
// save_checkpoint_secs=60) installs a CheckpointSaverHook whose Saver writes
// `model.ckpt-<step>.{index,data-XXXXX-of-YYYYY}` via the SaveV2/MergeV2Checkpoints kernels on
// the PS (/root/reference/distribute_training.py:204-215). This file is our native
// equivalent of those kernels:
//   * `<prefix>.data-<shard>-of-<num_shards>`: raw little-endian tensor bytes, concatenated
//     in insertion order;
//   * `<prefix>.index`: a LevelDB-format table (no compression, 16-entry restart interval,
//     256 KiB blocks) mapping "" -> BundleHeaderProto and each key -> BundleEntryProto.
// Entries carry the masked crc32c of their bytes, verified on read.
#include <algorithm>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "common.h"

namespace {

using ttd::put_fixed32;
using ttd::put_fixed64;
using ttd::put_varint32;
using ttd::put_varint64;

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr size_t kBlockSize = 262144;
constexpr int kRestartInterval = 16;
constexpr int kMaxEncodedHandle = 20;  // 2 x varint64 max
constexpr int kFooterLength = 2 * kMaxEncodedHandle + 8;
constexpr int kDtString = 7;

std::string shard_name(const std::string& prefix, int shard, int num) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), ".data-%05d-of-%05d", shard, num);
  return prefix + buf;
}

// ---------------------------------------------------------------- protobuf encoding
void pb_tag(std::string* s, int field, int wire) { put_varint32(s, (field << 3) | wire); }
void pb_varint(std::string* s, int field, uint64_t v) {
  if (v == 0) return;  // proto3 default omitted
  pb_tag(s, field, 0);
  put_varint64(s, v);
}
void pb_bytes(std::string* s, int field, const std::string& v) {
  pb_tag(s, field, 2);
  put_varint64(s, v.size());
  s->append(v);
}

struct Entry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard_id = 0;
  uint64_t offset = 0;
  uint64_t size = 0;
  uint32_t masked_crc = 0;
  std::string raw_slices;  // unparsed field 7 (kept for round-trip)

  std::string encode() const {
    std::string s;
    pb_varint(&s, 1, static_cast<uint64_t>(dtype));
    std::string shp;
    for (int64_t d : shape) {
      std::string dim;
      pb_varint(&dim, 1, static_cast<uint64_t>(d));
      pb_bytes(&shp, 2, dim);
    }
    pb_bytes(&s, 2, shp);  // message field: present even when empty (scalar)
    pb_varint(&s, 3, static_cast<uint64_t>(shard_id));
    pb_varint(&s, 4, offset);
    pb_varint(&s, 5, size);
    if (masked_crc) {
      pb_tag(&s, 6, 5);
      put_fixed32(&s, masked_crc);
    }
    s.append(raw_slices);
    return s;
  }
};

std::string encode_header(int num_shards) {
  std::string s;
  pb_varint(&s, 1, static_cast<uint64_t>(num_shards));
  // endianness LITTLE = 0 -> omitted; version { producer: 1 }
  std::string ver;
  pb_varint(&ver, 1, 1);
  pb_bytes(&s, 3, ver);
  return s;
}

// Minimal protobuf reader.
struct PbReader {
  const char* p;
  const char* end;
  bool next(int* field, int* wire) {
    if (p >= end) return false;
    uint64_t t;
    p = ttd::get_varint64(p, end, &t);
    if (!p) return false;
    *field = static_cast<int>(t >> 3);
    *wire = static_cast<int>(t & 7);
    return true;
  }
  bool varint(uint64_t* v) { return (p = ttd::get_varint64(p, end, v)) != nullptr; }
  bool bytes(const char** b, uint64_t* n) {
    if (!varint(n) || p + *n > end) return false;
    *b = p;
    p += *n;
    return true;
  }
  bool skip(int wire) {
    uint64_t v;
    const char* b;
    switch (wire) {
      case 0: return varint(&v);
      case 1: p += 8; return p <= end;
      case 2: return bytes(&b, &v);
      case 5: p += 4; return p <= end;
      default: return false;
    }
  }
};

bool decode_entry(const std::string& val, Entry* e) {
  PbReader r{val.data(), val.data() + val.size()};
  int f, w;
  while (r.next(&f, &w)) {
    uint64_t v;
    const char* b;
    uint64_t n;
    if (f == 1 && w == 0) { if (!r.varint(&v)) return false; e->dtype = static_cast<int>(v); }
    else if (f == 2 && w == 2) {
      if (!r.bytes(&b, &n)) return false;
      PbReader sr{b, b + n};
      int f2, w2;
      while (sr.next(&f2, &w2)) {
        if (f2 == 2 && w2 == 2) {
          const char* db; uint64_t dn;
          if (!sr.bytes(&db, &dn)) return false;
          PbReader dr{db, db + dn};
          int f3, w3; int64_t size = 0;
          while (dr.next(&f3, &w3)) {
            if (f3 == 1 && w3 == 0) { uint64_t dv; if (!dr.varint(&dv)) return false; size = static_cast<int64_t>(dv); }
            else if (!dr.skip(w3)) return false;
          }
          e->shape.push_back(size);
        } else if (!sr.skip(w2)) return false;
      }
    }
    else if (f == 3 && w == 0) { if (!r.varint(&v)) return false; e->shard_id = static_cast<int>(v); }
    else if (f == 4 && w == 0) { if (!r.varint(&v)) return false; e->offset = v; }
    else if (f == 5 && w == 0) { if (!r.varint(&v)) return false; e->size = v; }
    else if (f == 6 && w == 5) { if (r.p + 4 > r.end) return false; e->masked_crc = ttd::get_fixed32(r.p); r.p += 4; }
    else if (f == 7 && w == 2) {
      const char* start = r.p;
      // re-encode the raw field (tag + len + bytes) for round trip
      if (!r.bytes(&b, &n)) return false;
      std::string raw; pb_tag(&raw, 7, 2); put_varint64(&raw, n); raw.append(b, n);
      e->raw_slices += raw;
      (void)start;
    }
    else if (!r.skip(w)) return false;
  }
  return true;
}

int decode_header_num_shards(const std::string& val) {
  PbReader r{val.data(), val.data() + val.size()};
  int f, w;
  int num = 0;
  while (r.next(&f, &w)) {
    uint64_t v;
    if (f == 1 && w == 0) { if (!r.varint(&v)) return -1; num = static_cast<int>(v); }
    else if (!r.skip(w)) return -1;
  }
  return num;
}

// ---------------------------------------------------------------- LevelDB table
class BlockBuilder {
 public:
  explicit BlockBuilder(int restart_interval) : interval_(restart_interval) { restarts_.push_back(0); }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter_ < interval_) {
      const size_t mn = std::min(last_key_.size(), key.size());
      while (shared < mn && last_key_[shared] == key[shared]) ++shared;
    } else {
      restarts_.push_back(static_cast<uint32_t>(buf_.size()));
      counter_ = 0;
    }
    put_varint32(&buf_, static_cast<uint32_t>(shared));
    put_varint32(&buf_, static_cast<uint32_t>(key.size() - shared));
    put_varint32(&buf_, static_cast<uint32_t>(value.size()));
    buf_.append(key.data() + shared, key.size() - shared);
    buf_.append(value);
    last_key_ = key;
    ++counter_;
    empty_ = false;
  }
  size_t size_estimate() const { return buf_.size() + restarts_.size() * 4 + 4; }
  bool empty() const { return empty_; }
  std::string finish() {
    std::string out = buf_;
    for (uint32_t r : restarts_) put_fixed32(&out, r);
    put_fixed32(&out, static_cast<uint32_t>(restarts_.size()));
    return out;
  }
  void reset() {
    buf_.clear();
    restarts_.assign(1, 0);
    counter_ = 0;
    last_key_.clear();
    empty_ = true;
  }

 private:
  int interval_;
  std::string buf_;
  std::vector<uint32_t> restarts_;
  int counter_ = 0;
  std::string last_key_;
  bool empty_ = true;
};

void shortest_separator(std::string* start, const std::string& limit) {
  size_t mn = std::min(start->size(), limit.size());
  size_t i = 0;
  while (i < mn && (*start)[i] == limit[i]) ++i;
  if (i >= mn) return;
  uint8_t b = static_cast<uint8_t>((*start)[i]);
  if (b < 0xff && b + 1 < static_cast<uint8_t>(limit[i])) {
    (*start)[i] = static_cast<char>(b + 1);
    start->resize(i + 1);
  }
}

void short_successor(std::string* key) {
  for (size_t i = 0; i < key->size(); ++i) {
    uint8_t b = static_cast<uint8_t>((*key)[i]);
    if (b != 0xff) {
      (*key)[i] = static_cast<char>(b + 1);
      key->resize(i + 1);
      return;
    }
  }
}

void encode_handle(std::string* s, uint64_t off, uint64_t size) {
  put_varint64(s, off);
  put_varint64(s, size);
}

// Builds a complete table image in memory from sorted (key, value) pairs.
std::string build_table(const std::vector<std::pair<std::string, std::string>>& kv) {
  std::string file;
  BlockBuilder data(kRestartInterval), index(1);
  std::string last_key;
  bool pending = false;
  uint64_t pend_off = 0, pend_size = 0;
  auto write_block = [&](BlockBuilder* b, uint64_t* off, uint64_t* size) {
    std::string raw = b->finish();
    *off = file.size();
    *size = raw.size();
    file.append(raw);
    char type = 0;  // kNoCompression
    uint32_t crc = ttd::crc32c_extend(ttd::crc32c_value(raw.data(), raw.size()), &type, 1);
    file.push_back(type);
    put_fixed32(&file, ttd::crc32c_mask(crc));
    b->reset();
  };
  for (const auto& e : kv) {
    if (pending) {
      shortest_separator(&last_key, e.first);
      std::string h;
      encode_handle(&h, pend_off, pend_size);
      index.add(last_key, h);
      pending = false;
    }
    last_key = e.first;
    data.add(e.first, e.second);
    if (data.size_estimate() >= kBlockSize) {
      write_block(&data, &pend_off, &pend_size);
      pending = true;
    }
  }
  if (!data.empty()) {
    write_block(&data, &pend_off, &pend_size);
    pending = true;
  }
  BlockBuilder meta(kRestartInterval);
  uint64_t meta_off, meta_size;
  write_block(&meta, &meta_off, &meta_size);
  if (pending) {
    short_successor(&last_key);
    std::string h;
    encode_handle(&h, pend_off, pend_size);
    index.add(last_key, h);
  }
  uint64_t idx_off, idx_size;
  write_block(&index, &idx_off, &idx_size);
  std::string footer;
  encode_handle(&footer, meta_off, meta_size);
  encode_handle(&footer, idx_off, idx_size);
  footer.resize(2 * kMaxEncodedHandle, '\0');
  put_fixed32(&footer, static_cast<uint32_t>(kTableMagic & 0xffffffffu));
  put_fixed32(&footer, static_cast<uint32_t>(kTableMagic >> 32));
  file.append(footer);
  return file;
}

bool read_file(const std::string& path, std::string* out) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out->resize(static_cast<size_t>(n));
  bool ok = n == 0 || std::fread(&(*out)[0], 1, static_cast<size_t>(n), f) == static_cast<size_t>(n);
  std::fclose(f);
  return ok;
}

bool write_file(const std::string& path, const std::string& data) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = data.empty() || std::fwrite(data.data(), 1, data.size(), f) == data.size();
  ok = (std::fclose(f) == 0) && ok;
  return ok;
}

bool parse_block(const std::string& file, uint64_t off, uint64_t size,
                 std::vector<std::pair<std::string, std::string>>* out) {
  if (off + size + 5 > file.size()) return false;
  const char* b = file.data() + off;
  char type = b[size];
  uint32_t crc = ttd::crc32c_extend(ttd::crc32c_value(b, size), &type, 1);
  if (ttd::crc32c_mask(crc) != ttd::get_fixed32(b + size + 1)) {
    ttd::set_error("index block crc mismatch");
    return false;
  }
  if (type != 0) {
    ttd::set_error("compressed index blocks are not supported");
    return false;
  }
  if (size < 4) return false;
  uint32_t nrest = ttd::get_fixed32(b + size - 4);
  if (4ull * nrest + 4 > size) return false;
  const char* p = b;
  const char* limit = b + size - 4 - 4ull * nrest;
  std::string key;
  while (p < limit) {
    uint64_t shared, nonshared, vlen;
    if (!(p = ttd::get_varint64(p, limit, &shared))) return false;
    if (!(p = ttd::get_varint64(p, limit, &nonshared))) return false;
    if (!(p = ttd::get_varint64(p, limit, &vlen))) return false;
    if (p + nonshared + vlen > limit || shared > key.size()) return false;
    key.resize(shared);
    key.append(p, nonshared);
    p += nonshared;
    out->emplace_back(key, std::string(p, vlen));
    p += vlen;
  }
  return true;
}

bool parse_table(const std::string& file, std::vector<std::pair<std::string, std::string>>* kv) {
  if (file.size() < static_cast<size_t>(kFooterLength)) {
    ttd::set_error("index file too short");
    return false;
  }
  const char* ft = file.data() + file.size() - kFooterLength;
  uint64_t magic = static_cast<uint64_t>(ttd::get_fixed32(ft + 40)) |
                   (static_cast<uint64_t>(ttd::get_fixed32(ft + 44)) << 32);
  if (magic != kTableMagic) {
    ttd::set_error("bad table magic");
    return false;
  }
  const char* p = ft;
  const char* lim = ft + 40;
  uint64_t mo, ms, io, is;
  if (!(p = ttd::get_varint64(p, lim, &mo)) || !(p = ttd::get_varint64(p, lim, &ms)) ||
      !(p = ttd::get_varint64(p, lim, &io)) || !(p = ttd::get_varint64(p, lim, &is))) {
    ttd::set_error("bad footer");
    return false;
  }
  std::vector<std::pair<std::string, std::string>> index;
  if (!parse_block(file, io, is, &index)) return false;
  for (auto& ie : index) {
    const char* hp = ie.second.data();
    const char* hl = hp + ie.second.size();
    uint64_t bo, bs;
    if (!(hp = ttd::get_varint64(hp, hl, &bo)) || !(hp = ttd::get_varint64(hp, hl, &bs))) return false;
    if (!parse_block(file, bo, bs, kv)) return false;
  }
  return true;
}

// ---------------------------------------------------------------- writer
struct Writer {
  std::string prefix;
  std::string index_path;
  int shard_id = 0;
  int num_shards = 1;
  FILE* data = nullptr;
  uint64_t offset = 0;
  std::map<std::string, Entry> entries;
};

struct Reader {
  std::string prefix;
  int num_shards = 1;
  std::vector<std::string> keys;
  std::map<std::string, Entry> entries;
  std::vector<FILE*> shards;
};

}  // namespace

TTD_EXPORT void* ttd_bundle_writer_open(const char* prefix, int shard_id, int num_shards) {
  auto w = std::make_unique<Writer>();
  w->prefix = prefix;
  w->index_path = w->prefix + ".index";
  w->shard_id = shard_id;
  w->num_shards = num_shards;
  std::string dp = shard_name(w->prefix, shard_id, num_shards);
  w->data = std::fopen(dp.c_str(), "wb");
  if (!w->data) {
    ttd::set_error("cannot open data file " + dp);
    return nullptr;
  }
  return w.release();
}

TTD_EXPORT int ttd_bundle_writer_add(void* h, const char* key, int dtype, int ndims, const int64_t* shape,
                                     const void* data, uint64_t nbytes) {
  auto* w = static_cast<Writer*>(h);
  std::string k(key);
  if (k.empty() || w->entries.count(k)) {
    ttd::set_error("duplicate or empty key: " + k);
    return -1;
  }
  Entry e;
  e.dtype = dtype;
  e.shape.assign(shape, shape + ndims);
  e.shard_id = w->shard_id;
  e.offset = w->offset;
  e.size = nbytes;
  e.masked_crc = ttd::crc32c_mask(ttd::crc32c_value(data, nbytes));
  if (nbytes && std::fwrite(data, 1, nbytes, w->data) != nbytes) {
    ttd::set_error("data write failed");
    return -1;
  }
  w->offset += nbytes;
  w->entries.emplace(k, std::move(e));
  return 0;
}

// DT_STRING tensor: [varint64 len_i]* | uint32 masked crc32c(lengths) | bytes_i*.
TTD_EXPORT int ttd_bundle_writer_add_strings(void* h, const char* key, int ndims, const int64_t* shape, int n,
                                             const char* const* strs, const uint64_t* lens) {
  auto* w = static_cast<Writer*>(h);
  std::string buf;
  uint32_t crc = 0;
  for (int i = 0; i < n; ++i) {
    std::string l;
    put_varint64(&l, lens[i]);
    crc = ttd::crc32c_extend(crc, l.data(), l.size());
    buf.append(l);
  }
  uint32_t lck = ttd::crc32c_mask(crc);
  put_fixed32(&buf, lck);
  crc = ttd::crc32c_extend(crc, &lck, 4);
  for (int i = 0; i < n; ++i) {
    buf.append(strs[i], lens[i]);
    crc = ttd::crc32c_extend(crc, strs[i], lens[i]);
  }
  std::string k(key);
  Entry e;
  e.dtype = kDtString;
  e.shape.assign(shape, shape + ndims);
  e.shard_id = w->shard_id;
  e.offset = w->offset;
  e.size = buf.size();
  e.masked_crc = ttd::crc32c_mask(crc);
  if (!buf.empty() && std::fwrite(buf.data(), 1, buf.size(), w->data) != buf.size()) {
    ttd::set_error("data write failed");
    return -1;
  }
  w->offset += buf.size();
  w->entries.emplace(k, std::move(e));
  return 0;
}

TTD_EXPORT int ttd_bundle_writer_finish(void* h) {
  std::unique_ptr<Writer> w(static_cast<Writer*>(h));
  if (std::fclose(w->data) != 0) {
    ttd::set_error("data close failed");
    return -1;
  }
  std::vector<std::pair<std::string, std::string>> kv;
  kv.emplace_back("", encode_header(w->num_shards));
  for (auto& e : w->entries) kv.emplace_back(e.first, e.second.encode());
  if (!write_file(w->index_path, build_table(kv))) {
    ttd::set_error("cannot write " + w->index_path);
    return -1;
  }
  return 0;
}

// MergeV2Checkpoints equivalent: `n` single-shard bundles (each written with
// shard_id=0,num_shards=1) become one n-shard bundle at out_prefix. Data files are
// renamed to out_prefix.data-k-of-n; the partial indices are removed.
TTD_EXPORT int ttd_bundle_merge(int n, const char* const* in_prefixes, const char* out_prefix) {
  std::map<std::string, Entry> merged;
  for (int k = 0; k < n; ++k) {
    std::string ip = std::string(in_prefixes[k]) + ".index";
    std::string file;
    if (!read_file(ip, &file)) {
      ttd::set_error("cannot read " + ip);
      return -1;
    }
    std::vector<std::pair<std::string, std::string>> kv;
    if (!parse_table(file, &kv)) return -1;
    for (auto& e : kv) {
      if (e.first.empty()) continue;
      Entry en;
      if (!decode_entry(e.second, &en)) {
        ttd::set_error("bad entry " + e.first);
        return -1;
      }
      en.shard_id = k;
      if (!merged.emplace(e.first, en).second) {
        ttd::set_error("duplicate key across shards: " + e.first);
        return -1;
      }
    }
    std::string src = shard_name(in_prefixes[k], 0, 1);
    std::string dst = shard_name(out_prefix, k, n);
    if (std::rename(src.c_str(), dst.c_str()) != 0) {
      ttd::set_error("rename failed: " + src + " -> " + dst);
      return -1;
    }
    std::remove(ip.c_str());
  }
  std::vector<std::pair<std::string, std::string>> kv;
  kv.emplace_back("", encode_header(n));
  for (auto& e : merged) kv.emplace_back(e.first, e.second.encode());
  std::string op = std::string(out_prefix) + ".index";
  if (!write_file(op, build_table(kv))) {
    ttd::set_error("cannot write " + op);
    return -1;
  }
  return 0;
}

TTD_EXPORT void* ttd_bundle_reader_open(const char* prefix) {
  auto r = std::make_unique<Reader>();
  r->prefix = prefix;
  std::string file;
  if (!read_file(r->prefix + ".index", &file)) {
    ttd::set_error("cannot read " + r->prefix + ".index");
    return nullptr;
  }
  std::vector<std::pair<std::string, std::string>> kv;
  if (!parse_table(file, &kv)) return nullptr;
  for (auto& e : kv) {
    if (e.first.empty()) {
      r->num_shards = decode_header_num_shards(e.second);
      continue;
    }
    Entry en;
    if (!decode_entry(e.second, &en)) {
      ttd::set_error("bad entry " + e.first);
      return nullptr;
    }
    r->keys.push_back(e.first);
    r->entries.emplace(e.first, en);
  }
  r->shards.assign(static_cast<size_t>(std::max(r->num_shards, 1)), nullptr);
  return r.release();
}

TTD_EXPORT int ttd_bundle_reader_num_entries(void* h) { return static_cast<int>(static_cast<Reader*>(h)->keys.size()); }
TTD_EXPORT int ttd_bundle_reader_num_shards(void* h) { return static_cast<Reader*>(h)->num_shards; }
TTD_EXPORT const char* ttd_bundle_reader_key(void* h, int i) { return static_cast<Reader*>(h)->keys[i].c_str(); }

// shape must have room for 32 dims. Returns ndims, or -1 if key missing.
TTD_EXPORT int ttd_bundle_reader_entry(void* h, const char* key, int* dtype, int64_t* shape, uint64_t* nbytes,
                                       int* shard_id, uint64_t* offset, uint32_t* masked_crc) {
  auto* r = static_cast<Reader*>(h);
  auto it = r->entries.find(key);
  if (it == r->entries.end()) {
    ttd::set_error(std::string("key not found: ") + key);
    return -1;
  }
  const Entry& e = it->second;
  *dtype = e.dtype;
  int nd = static_cast<int>(std::min<size_t>(e.shape.size(), 32));
  for (int i = 0; i < nd; ++i) shape[i] = e.shape[i];
  *nbytes = e.size;
  if (shard_id) *shard_id = e.shard_id;
  if (offset) *offset = e.offset;
  if (masked_crc) *masked_crc = e.masked_crc;
  return nd;
}

// Reads the raw entry bytes (for DT_STRING this is the length-prefixed encoding) and
// verifies the masked crc32c.
TTD_EXPORT int ttd_bundle_reader_read(void* h, const char* key, void* out, uint64_t nbytes) {
  auto* r = static_cast<Reader*>(h);
  auto it = r->entries.find(key);
  if (it == r->entries.end()) {
    ttd::set_error(std::string("key not found: ") + key);
    return -1;
  }
  const Entry& e = it->second;
  if (nbytes != e.size) {
    ttd::set_error("size mismatch for " + std::string(key));
    return -1;
  }
  if (e.shard_id < 0 || e.shard_id >= static_cast<int>(r->shards.size())) {
    ttd::set_error("bad shard id");
    return -1;
  }
  FILE*& f = r->shards[e.shard_id];
  if (!f) {
    std::string dp = shard_name(r->prefix, e.shard_id, r->num_shards);
    f = std::fopen(dp.c_str(), "rb");
    if (!f) {
      ttd::set_error("cannot open " + dp);
      return -1;
    }
  }
  if (std::fseek(f, static_cast<long>(e.offset), SEEK_SET) != 0 ||
      (nbytes && std::fread(out, 1, nbytes, f) != nbytes)) {
    ttd::set_error("short read for " + std::string(key));
    return -1;
  }
  if (ttd::crc32c_mask(ttd::crc32c_value(out, nbytes)) != e.masked_crc) {
    ttd::set_error("crc32c mismatch for " + std::string(key));
    return -2;
  }
  return 0;
}

TTD_EXPORT void ttd_bundle_reader_close(void* h) {
  auto* r = static_cast<Reader*>(h);
  if (!r) return;
  for (FILE* f : r->shards)
    if (f) std::fclose(f);
  delete r;
}
