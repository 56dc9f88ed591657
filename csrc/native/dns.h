// DNS query-name feature extraction (see dns.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace onin {

struct DnsFeatures {
  std::vector<int32_t> domain_id, sub_id, sub_len, num_parts;
  std::vector<double> entropy;
  std::vector<int8_t> top;
  std::vector<std::string> domains, subs;
};

double scala_entropy(std::string_view s);
void java_split_dot(std::string_view s, std::vector<std::string_view>& parts);
DnsFeatures dns_features(const char* data, const int64_t* offsets, int64_t n, const std::vector<std::string>& cc,
                         const std::vector<std::string>& top, const std::string& special, int threads);

}  // namespace onin
