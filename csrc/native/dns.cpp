// DNS query-name features (reference: dns_pre_lda.scala:185-227,278-287,313-316;
// SURVEY.md C6d/C6e/C6g, hot op H14).  Multithreaded over names.
//
// extract_subdomain(url):
//   parts = url.split("[.]")  (Java: trailing empty labels dropped; "" -> [""])
//   if #parts > 2 and not *.in-addr.arpa:
//     last label in country-code set -> domain = parts[n-3], subdomain = parts[0, n-3) joined by '.'
//     else                            -> domain = parts[n-2], subdomain = parts[0, n-2)
//   defaults "None"; subdomain.length = UTF-16 length of subdomain (0 for "None");
//   num.periods = #parts (the label count).
// entropy(subdomain) = sum over distinct chars of -p*log10(p)/log10(2), the
//   sum taken in the iteration order of the Scala 2.10 `groupBy` Map the
//   reference builds (see scala_group_order), so equal inputs give equal bits.
// top_domain = "2" if domain == "intel", "1" if domain in the top-1m first-label
//   set, else "0".
#include "dns.h"

#include <algorithm>
#include <cmath>
#include <thread>
#include <unordered_map>
#include <unordered_set>

namespace onin {

namespace {

// UTF-8 -> UTF-16 code units (what Java's String holds).
void utf16_units(std::string_view s, std::vector<uint16_t>& out) {
  out.clear();
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); n = 2; }
    else if ((c >> 4) == 14 && i + 2 < s.size()) {
      cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); n = 3;
    } else if ((c >> 3) == 30 && i + 3 < s.size()) {
      cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F); n = 4;
    } else { cp = 0xFFFD; n = 1; }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      out.push_back((uint16_t)(0xD800 + (cp >> 10)));
      out.push_back((uint16_t)(0xDC00 + (cp & 0x3FF)));
    } else {
      out.push_back((uint16_t)cp);
    }
    i += n;
  }
}

inline int32_t byteswap32(int32_t v) {
  uint32_t hc = (uint32_t)v * 0x9e3775cdu;
  hc = __builtin_bswap32(hc);
  return (int32_t)(hc * 0x9e3775cdu);
}

// scala.collection.mutable.HashTable bucket of a key in a 16-slot table.
inline int mutable_bucket(int32_t h) {
  uint32_t i = (uint32_t)byteswap32(h);
  const int rot = 4;  // tableSizeSeed = bitCount(15)
  uint32_t r = (i >> rot) | (i << (32 - rot));
  return (int)(((int32_t)r >> (32 - 4)) & 15);
}

// scala.collection.immutable.HashMap.improve
inline uint32_t immutable_improve(int32_t hcode) {
  int32_t h = hcode + ~(hcode << 9);
  h = h ^ (int32_t)((uint32_t)h >> 14);
  h = h + (h << 4);
  return (uint32_t)(h ^ (int32_t)((uint32_t)h >> 10));
}

// Order in which `s.groupBy(c => c).values` yields the groups under Scala 2.10:
// groupBy fills a mutable.HashMap (16 buckets, chained by prepending) and then
// copies it, in that map's iteration order (buckets high -> low), into an
// immutable Map: Map1..Map4 keep that order, a 5th key turns it into a
// HashTrieMap iterated by the 5-bit chunks of the improved hash, low bits first.
void scala_group_order(const std::vector<uint16_t>& u, std::vector<uint16_t>& keys, std::vector<int>& cnt) {
  keys.clear();
  cnt.clear();
  std::vector<uint16_t> first;  // first-appearance order
  std::unordered_map<uint16_t, int> c;
  for (uint16_t x : u) {
    auto it = c.find(x);
    if (it == c.end()) { c.emplace(x, 1); first.push_back(x); }
    else ++it->second;
  }
  const size_t n = first.size();
  if (n <= 4) {
    // mutable map iteration: bucket descending; within a bucket newest first
    std::vector<std::pair<int, int>> ord;  // (bucket, insertion rank)
    for (size_t i = 0; i < n; ++i) ord.emplace_back(mutable_bucket((int32_t)first[i]), (int)i);
    std::sort(ord.begin(), ord.end(), [](auto a, auto b) {
      if (a.first != b.first) return a.first > b.first;
      return a.second > b.second;
    });
    for (auto& p : ord) { keys.push_back(first[p.second]); cnt.push_back(c[first[p.second]]); }
    return;
  }
  std::vector<std::pair<uint64_t, uint16_t>> ord;
  for (uint16_t x : first) {
    uint32_t h = immutable_improve((int32_t)x);
    // lexicographic on (h & 31, h >> 5 & 31, ...) == numeric order of the 5-bit-chunk-reversed hash
    uint64_t key = 0;
    for (int lvl = 0; lvl < 7; ++lvl) key = (key << 5) | ((h >> (5 * lvl)) & 31u);
    ord.emplace_back(key, x);
  }
  std::sort(ord.begin(), ord.end());
  for (auto& p : ord) { keys.push_back(p.second); cnt.push_back(c[p.second]); }
}

struct LocalDict {
  std::vector<std::string> names;
  std::unordered_map<std::string, int32_t> index;
  int32_t add(const std::string& s) {
    auto it = index.find(s);
    if (it != index.end()) return it->second;
    int32_t id = (int32_t)names.size();
    names.push_back(s);
    index.emplace(s, id);
    return id;
  }
};

}  // namespace

double scala_entropy(std::string_view s) {
  std::vector<uint16_t> u, keys;
  std::vector<int> cnt;
  utf16_units(s, u);
  scala_group_order(u, keys, cnt);
  const double len = (double)u.size();
  const double l2 = std::log10(2.0);
  double sum = 0.0;
  for (int k : cnt) {
    const double p = (double)k / len;
    sum = sum + (-p * std::log10(p) / l2);
  }
  return sum;
}

void java_split_dot(std::string_view s, std::vector<std::string_view>& parts) {
  parts.clear();
  if (s.empty()) { parts.push_back(s); return; }
  size_t b = 0;
  for (size_t i = 0; i <= s.size(); ++i) {
    if (i == s.size() || s[i] == '.') {
      parts.push_back(s.substr(b, i - b));
      b = i + 1;
    }
  }
  while (!parts.empty() && parts.back().empty()) parts.pop_back();
}

DnsFeatures dns_features(const char* data, const int64_t* offsets, int64_t n, const std::vector<std::string>& cc,
                         const std::vector<std::string>& top, const std::string& special, int threads) {
  std::unordered_set<std::string> ccset(cc.begin(), cc.end()), topset(top.begin(), top.end());
  DnsFeatures F;
  F.sub_len.resize(n);
  F.num_parts.resize(n);
  F.entropy.resize(n);
  F.top.resize(n);
  F.domain_id.resize(n);
  F.sub_id.resize(n);
  if (threads < 1) threads = 1;
  if (n < 65536) threads = 1;
  std::vector<LocalDict> ldom(threads), lsub(threads);
  auto work = [&](int t) {
    const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    std::vector<std::string_view> parts;
    std::vector<uint16_t> u;
    std::string sub;
    for (int64_t i = lo; i < hi; ++i) {
      std::string_view url(data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
      java_split_dot(url, parts);
      const int np = (int)parts.size();
      std::string domain = "None";
      sub = "None";
      bool is_ip = np > 2 && parts[np - 1] == "arpa" && parts[np - 2] == "in-addr";
      if (np > 2 && !is_ip) {
        int cut = ccset.count(std::string(parts[np - 1])) ? np - 3 : np - 2;
        domain = std::string(parts[cut]);
        if (1 <= cut) {
          sub.clear();
          for (int j = 0; j < cut; ++j) {
            if (j) sub += '.';
            sub.append(parts[j].data(), parts[j].size());
          }
        }
      }
      utf16_units(sub, u);
      F.sub_len[i] = sub == "None" ? 0 : (int32_t)u.size();
      F.num_parts[i] = np;
      F.entropy[i] = scala_entropy(sub);
      F.top[i] = domain == special ? 2 : (topset.count(domain) ? 1 : 0);
      F.domain_id[i] = ldom[t].add(domain);
      F.sub_id[i] = lsub[t].add(sub);
    }
  };
  if (threads == 1) work(0);
  else {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  LocalDict gd, gs;
  for (int t = 0; t < threads; ++t) {
    const int64_t lo = n * t / threads, hi = n * (t + 1) / threads;
    std::vector<int32_t> rd(ldom[t].names.size()), rs(lsub[t].names.size());
    for (size_t j = 0; j < rd.size(); ++j) rd[j] = gd.add(ldom[t].names[j]);
    for (size_t j = 0; j < rs.size(); ++j) rs[j] = gs.add(lsub[t].names[j]);
    for (int64_t i = lo; i < hi; ++i) {
      F.domain_id[i] = rd[F.domain_id[i]];
      F.sub_id[i] = rs[F.sub_id[i]];
    }
  }
  F.domains = std::move(gd.names);
  F.subs = std::move(gs.names);
  return F;
}

}  // namespace onin
