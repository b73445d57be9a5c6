// Flow-text ingest: ovs-ofctl flow text -> realized flow table.
//
// Accepts the text FlowModToString prints (pkg/ovs/openflow/utils.go:1222-1241, with the match
// field order of getFlowModMatch :905-1098 and the action forms of :600-760) and the lines
// `ovs-ofctl dump-flows --names` prints for the same flows (cookie / duration / n_packets /
// n_bytes / idle_age fields, `resubmit(,T)`), i.e. what Antrea's agent hands to
// Bridge.AddFlowsInBundle (pkg/ovs/openflow/ofctrl_bridge.go:468) and what
// network_policy.go:1948 parseFlowToMap reads back. Flows of tables outside the NetworkPolicy
// path are skipped (counted), so a whole-bridge dump can be loaded.
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "compiler.hpp"
#include "model.hpp"

namespace gpc {

namespace {

// Splits on `sep` at parenthesis depth 0.
std::vector<std::string> split_top(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  int depth = 0;
  for (char ch : s) {
    if (ch == '(') depth++;
    if (ch == ')') depth--;
    if (ch == sep && depth == 0) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += ch;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

bool num(const std::string& s, unsigned long long* v) {
  if (s.empty()) return false;
  char* end = nullptr;
  *v = std::strtoull(s.c_str(), &end, 0);
  return end && *end == 0;
}

bool value_mask(const std::string& s, unsigned long long* v, unsigned long long* m, bool* has_mask) {
  size_t p = s.find('/');
  *has_mask = p != std::string::npos;
  if (!*has_mask) return num(s, v);
  return num(s.substr(0, p), v) && num(s.substr(p + 1), m);
}

int table_id(const std::string& name) {
  for (int t = 1; t < TB_COUNT; t++)
    if (name == table_name(uint8_t(t))) return t;
  return -1;
}

bool parse_ip(const std::string& s, IPMatch* m) {
  std::string a = s;
  int plen = -1;
  size_t p = s.find('/');
  if (p != std::string::npos) {
    a = s.substr(0, p);
    char* end = nullptr;
    long l = std::strtol(s.c_str() + p + 1, &end, 10);
    if (!end || *end) return false;
    plen = int(l);
  }
  IPAddr ip;
  if (a.find(':') == std::string::npos) {
    unsigned b[4];
    char tail;
    if (std::sscanf(a.c_str(), "%u.%u.%u.%u%c", &b[0], &b[1], &b[2], &b[3], &tail) != 4) return false;
    ip.fam = 4;
    for (int i = 0; i < 4; i++) {
      if (b[i] > 255) return false;
      ip.b[i] = uint8_t(b[i]);
    }
    if (plen > 32) return false;
  } else {  // IPv6: groups with at most one "::"
    ip.fam = 6;
    std::vector<std::string> head, tail;
    size_t dc = a.find("::");
    auto groups = [](const std::string& x, std::vector<std::string>* g) {
      size_t st = 0;
      while (st <= x.size() && !x.empty()) {
        size_t e = x.find(':', st);
        g->push_back(x.substr(st, e == std::string::npos ? std::string::npos : e - st));
        if (e == std::string::npos) break;
        st = e + 1;
      }
    };
    if (dc == std::string::npos) {
      groups(a, &head);
      if (head.size() != 8) return false;
    } else {
      groups(a.substr(0, dc), &head);
      groups(a.substr(dc + 2), &tail);
      if (head.size() + tail.size() > 7) return false;
    }
    std::vector<std::string> all = head;
    for (size_t i = head.size() + tail.size(); i < 8; i++) all.push_back("0");
    all.insert(all.end(), tail.begin(), tail.end());
    for (int i = 0; i < 8; i++) {
      char* end = nullptr;
      unsigned long g = std::strtoul(all[i].c_str(), &end, 16);
      if (all[i].empty() || !end || *end || g > 0xffff) return false;
      ip.b[2 * i] = uint8_t(g >> 8);
      ip.b[2 * i + 1] = uint8_t(g);
    }
    if (plen > 128) return false;
  }
  m->set = true;
  m->addr = ip;
  m->plen = plen;
  return true;
}

bool proto_word(const std::string& w, Match* m) {
  static const struct {
    const char* w;
    uint16_t eth;
    int proto;
  } kWords[] = {{"ip", kEthIP, -1},     {"ipv6", kEthIPv6, -1}, {"arp", 0x0806, -1},   {"tcp", kEthIP, 6},
                {"tcp6", kEthIPv6, 6},  {"udp", kEthIP, 17},    {"udp6", kEthIPv6, 17}, {"sctp", kEthIP, 132},
                {"sctp6", kEthIPv6, 132}, {"icmp", kEthIP, 1},  {"icmp6", kEthIPv6, 58}, {"igmp", kEthIP, 2}};
  for (auto& k : kWords)
    if (w == k.w) {
      m->has_dl = true;
      m->dl_type = k.eth;
      if (k.proto >= 0) {
        m->has_proto = true;
        m->nw_proto = uint8_t(k.proto);
      }
      return true;
    }
  return false;
}

bool parse_action(const std::string& a, Action* out) {
  unsigned long long v, m;
  bool hm;
  if (a == "drop") {
    *out = Action{ACT_DROP};
    return true;
  }
  if (a.compare(0, 12, "conjunction(") == 0) {
    unsigned id, k, n;
    if (std::sscanf(a.c_str(), "conjunction(%u,%u/%u)", &id, &k, &n) != 3) return false;
    *out = Action{ACT_CONJ};
    out->a = id;
    out->b = k;
    out->c = n;
    return true;
  }
  if (a.compare(0, 10, "set_field:") == 0) {
    size_t arrow = a.find("->");
    if (arrow == std::string::npos) return false;
    std::string dst = a.substr(arrow + 2);
    if (dst.compare(0, 3, "reg") != 0 || !value_mask(a.substr(10, arrow - 10), &v, &m, &hm)) return false;
    unsigned long long r;
    if (!num(dst.substr(3), &r) || r > 15) return false;
    *out = Action{ACT_SET_REG};
    out->a = uint32_t(r);
    out->b = uint32_t(v);
    out->c = hm ? uint32_t(m) : 0xffffffffu;
    out->has_mask = hm;
    return true;
  }
  if (a.compare(0, 3, "ct(") == 0 && a.back() == ')') {
    *out = Action{ACT_CT_COMMIT};
    bool commit = false;
    for (auto& part : split_top(a.substr(3, a.size() - 4), ',')) {
      if (part == "commit") {
        commit = true;
      } else if (part.compare(0, 6, "table=") == 0) {
        int t = table_id(part.substr(6));
        if (t < 0) return false;
        out->a = uint32_t(t);
      } else if (part.compare(0, 5, "zone=") == 0) {
        if (!num(part.substr(5), &v)) return false;
        out->b = uint32_t(v);
      } else if (part.compare(0, 5, "exec(") == 0 && part.back() == ')') {
        for (auto& ea : split_top(part.substr(5, part.size() - 6), ',')) {
          size_t arrow = ea.find("->ct_label");
          if (ea.compare(0, 10, "set_field:") != 0 || arrow == std::string::npos) return false;
          if (!value_mask(ea.substr(10, arrow - 10), &v, &m, &hm)) return false;
          out->lv = v;
          out->lm = hm ? m : ~0ull;
        }
      } else {
        return false;
      }
    }
    return commit;
  }
  std::string t;
  if (a.compare(0, 11, "goto_table:") == 0) t = a.substr(11);
  else if (a.compare(0, 10, "resubmit(,") == 0 && a.back() == ')') t = a.substr(10, a.size() - 11);
  else if (a.compare(0, 9, "resubmit:") == 0) t = a.substr(9);
  if (!t.empty()) {
    int id = table_id(t);
    if (id < 0) return false;
    *out = Action{ACT_GOTO};
    out->a = uint32_t(id);
    return true;
  }
  if (a.compare(0, 6, "group:") == 0) {
    if (!num(a.substr(6), &v)) return false;
    *out = Action{ACT_GROUP};
    out->a = uint32_t(v);
    return true;
  }
  if (a.compare(0, 6, "meter:") == 0) {
    if (!num(a.substr(6), &v)) return false;
    *out = Action{ACT_METER};
    out->a = uint32_t(v);
    return true;
  }
  if (a.compare(0, 11, "controller(") == 0 && a.back() == ')') {  // utils.go:800-838 (userdata kept, <= 4 bytes)
    *out = Action{ACT_CONTROLLER};
    for (auto& part : split_top(a.substr(11, a.size() - 12), ',')) {
      if (part.compare(0, 9, "userdata=") != 0) continue;
      uint32_t n = 0, packed = 0;
      for (auto& b : split_top(part.substr(9), '.')) {
        char* end = nullptr;
        unsigned long x = std::strtoul(b.c_str(), &end, 16);
        if (b.empty() || !end || *end || x > 255 || n >= 4) return false;
        packed |= uint32_t(x) << (8 * n++);
      }
      out->a = n;
      out->b = packed;
    }
    return true;
  }
  return false;
}

int bad_value(const std::string& k, const std::string& v, std::string* err) {
  *err = "bad value '" + v + "' for " + k;
  return -GPC_EINVAL;
}

}  // namespace

// Returns 1 (flow parsed), 0 (line skipped: blank, header, or a table outside the NP path) or
// -GPC_EINVAL with `err` set.
int parse_flow_text(const std::string& line_in, Flow* f, std::string* err) {
  std::string line = trim(line_in);
  if (line.empty() || line[0] == '#' || line.compare(0, 9, "NXST_FLOW") == 0 || line.compare(0, 10, "OFPST_FLOW") == 0)
    return 0;
  size_t ap = line.find(" actions=");
  if (ap == std::string::npos) {
    *err = "no actions: " + line;
    return -GPC_EINVAL;
  }
  *f = Flow();
  f->priority = 32768;
  bool have_table = false;
  Match& m = f->m;
  for (auto tok : split_top(line.substr(0, ap), ',')) {
    tok = trim(tok);
    if (tok.empty()) continue;
    size_t eq = tok.find('=');
    if (eq == std::string::npos) {
      if (!proto_word(tok, &m)) {
        *err = "unsupported match word '" + tok + "'";
        return -GPC_EINVAL;
      }
      continue;
    }
    std::string k = tok.substr(0, eq), v = tok.substr(eq + 1);
    unsigned long long x, y;
    bool hm;
    if (k == "table") {
      int t = table_id(v);
      // the NetworkPolicy tables, plus IngressSecurityClassifier and the packet-in flows of Output
      // (initFlows, network_policy.go:2126-2142); any other table is not on this path
      if (t < 0 || (t > TB_INGRESS_METRIC && t != TB_INGRESS_CLASSIFIER && t != TB_OUTPUT)) return 0;
      f->table = uint8_t(t);
      have_table = true;
    } else if (k == "priority") {
      if (!num(v, &x) || x > 65535) return bad_value(k, v, err);
      f->priority = uint16_t(x);
    } else if (k == "cookie") {
      if (!num(v.substr(0, v.find('/')), &x)) return bad_value(k, v, err);
      f->cookie = x;
    } else if (k == "duration" || k == "n_packets" || k == "n_bytes" || k == "idle_age" || k == "hard_age" ||
               k == "idle_timeout" || k == "hard_timeout" || k == "reset_counts") {
      continue;
    } else if (k == "conj_id") {
      if (!num(v, &x)) return bad_value(k, v, err);
      m.has_conj = true;
      m.conj_id = uint32_t(x);
    } else if (k == "ct_state") {
      static const char* cts[8] = {"new", "est", "rel", "rpl", "inv", "trk", "snat", "dnat"};
      m.has_ct_state = true;
      size_t i = 0;
      while (i < v.size()) {
        char sign = v[i++];
        size_t j = i;
        while (j < v.size() && v[j] != '+' && v[j] != '-') j++;
        std::string nm = v.substr(i, j - i);
        int bit = -1;
        for (int b = 0; b < 8; b++)
          if (nm == cts[b]) bit = b;
        if (bit < 0 || (sign != '+' && sign != '-')) {
          *err = "bad ct_state '" + v + "'";
          return -GPC_EINVAL;
        }
        m.ct_mask |= uint8_t(1u << bit);
        if (sign == '+') m.ct_data |= uint8_t(1u << bit);
        i = j;
      }
    } else if (k == "ct_mark") {
      if (!value_mask(v, &x, &y, &hm)) return bad_value(k, v, err);
      m.has_ct_mark = true;
      m.ct_mark_v = uint32_t(x);
      m.ct_mark_m = hm ? uint32_t(y) : 0xffffffffu;
    } else if (k == "ct_label") {
      if (!value_mask(v, &x, &y, &hm)) return bad_value(k, v, err);
      m.has_ct_label = true;
      m.label_v = x;
      m.label_m = hm ? y : ~0ull;
    } else if (k == "nw_src" || k == "ipv6_src") {
      if (!parse_ip(v, &m.nw_src)) return bad_value(k, v, err);
    } else if (k == "nw_dst" || k == "ipv6_dst") {
      if (!parse_ip(v, &m.nw_dst)) return bad_value(k, v, err);
    } else if (k == "ct_nw_src" || k == "ct_ipv6_src") {
      if (!parse_ip(v, &m.ct_nw_src)) return bad_value(k, v, err);
    } else if (k == "ct_nw_dst" || k == "ct_ipv6_dst") {
      if (!parse_ip(v, &m.ct_nw_dst)) return bad_value(k, v, err);
    } else if (k.size() > 3 && k.compare(0, 3, "reg") == 0) {
      unsigned long long r;
      if (!num(k.substr(3), &r) || r > 15 || !value_mask(v, &x, &y, &hm)) return bad_value(k, v, err);
      m.set_reg(int(r), uint32_t(x), hm ? uint32_t(y) : 0xffffffffu);
    } else if (k == "tun_id") {
      if (!num(v, &x)) return bad_value(k, v, err);
      m.has_tun = true;
      m.tun_id = x;
    } else if (k == "in_port") {
      if (!num(v, &x)) return bad_value(k, v, err);
      m.has_in_port = true;
      m.in_port = uint32_t(x);
    } else if (k == "icmp_type" || k == "icmpv6_type") {
      if (!num(v, &x)) return bad_value(k, v, err);
      m.has_icmp_type = true;
      m.icmp_type = uint8_t(x);
    } else if (k == "icmp_code" || k == "icmpv6_code") {
      if (!num(v, &x)) return bad_value(k, v, err);
      m.has_icmp_code = true;
      m.icmp_code = uint8_t(x);
    } else if (k == "tp_src" || k == "tp_dst") {
      if (!value_mask(v, &x, &y, &hm)) return bad_value(k, v, err);
      bool dst = k == "tp_dst";
      (dst ? m.has_tp_dst : m.has_tp_src) = true;
      (dst ? m.tp_dst : m.tp_src) = uint16_t(x);
      (dst ? m.tp_dst_m : m.tp_src_m) = hm ? uint16_t(y) : uint16_t(0xffff);
    } else {
      *err = "unsupported match field '" + k + "'";
      return -GPC_EINVAL;
    }
    continue;
  }
  if (!have_table) {
    *err = "no table: " + line;
    return -GPC_EINVAL;
  }
  for (auto a : split_top(line.substr(ap + 9), ',')) {
    a = trim(a);
    if (a.empty()) continue;
    Action act{ACT_DROP};
    if (!parse_action(a, &act)) {
      if (f->table == TB_OUTPUT) return 0;  // an Output flow of another feature
      *err = "unsupported action '" + a + "'";
      return -GPC_EINVAL;
    }
    f->acts.push_back(act);
  }
  return 1;
}

}  // namespace gpc
