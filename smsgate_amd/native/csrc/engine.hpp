// Broker state machine of the native bus daemon: streams, retention, durable
// competing consumers.  Semantics are those of the Python engine
// (smsgate_amd/bus/engine.py), which is the specification; the differential
// test (tests/test_native_bus.py) drives both with the same operations.
//
// Messages of a stream live in a deque indexed by ``seq - base`` (retention
// only ever drops from the front, so the live range stays dense); each
// consumer keeps a cursor, an unordered pending map (seq -> deadline,
// deliveries) and a lazily-invalidated min-heap of redelivery deadlines.
// Every mutation is reported through ``journal`` as (kind, args) in the same
// record shapes as smsgate_amd/bus/filelog.py, so either broker can recover
// the other's journal.
#pragma once

#include <algorithm>
#include <cmath>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "mpack.hpp"

namespace bus {

struct BusError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline std::vector<std::string> split_tokens(const std::string& s) {
  std::vector<std::string> out;
  size_t start = 0;
  for (;;) {
    size_t dot = s.find('.', start);
    out.emplace_back(s.substr(start, dot == std::string::npos ? std::string::npos : dot - start));
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return out;
}

// NATS-style: ``*`` = one token, ``>`` = one or more trailing tokens (base.py:132-145).
// Walks both strings token by token without allocating (the NATS front-end matches
// every routed message against every subscription).
inline bool subject_matches(const std::string& pattern, const std::string& subject) {
  if (pattern == subject) return true;
  const size_t P = pattern.size(), S = subject.size();
  size_t i = 0, j = 0;
  for (;;) {
    size_t pe = pattern.find('.', i);
    if (pe == std::string::npos) pe = P;
    const size_t pl = pe - i;
    if (pl == 1 && pattern[i] == '>') return j <= S;  // >= 1 subject token left
    if (j > S) return false;                          // subject has fewer tokens
    size_t se = subject.find('.', j);
    if (se == std::string::npos) se = S;
    if (!(pl == 1 && pattern[i] == '*') && (pl != se - j || pattern.compare(i, pl, subject, j, pl) != 0))
      return false;
    const bool pend = pe == P, send = se == S;
    if (pend || send) return pend && send;
    i = pe + 1;
    j = se + 1;
  }
}

struct StreamConfig {
  std::string name;
  std::vector<std::string> subjects;
  double max_age = 0.0;
  int64_t max_msgs = -1;
  int64_t max_bytes = -1;
  std::string storage = "file";
};

struct ConsumerConfig {
  std::string durable;
  std::string filter_subject = ">";
  double ack_wait = 30.0;
  int64_t max_deliver = -1;
  std::string deliver_policy = "all";
  int64_t max_ack_pending = 65536;
};

struct Stored {
  int64_t seq;
  std::string subject;
  std::string data;
  double ts;
  mp::Value headers;  // nil or a str->str map, kept opaque
};

struct Delivery {
  const Stored* msg;
  int64_t num_delivered;
};

struct Pending {
  double deadline;
  int64_t delivered;
};

struct Consumer {
  ConsumerConfig cfg;
  int64_t cursor = 0;
  std::unordered_map<int64_t, Pending> pending;
  std::priority_queue<std::pair<double, int64_t>, std::vector<std::pair<double, int64_t>>,
                      std::greater<std::pair<double, int64_t>>> heap;
  int64_t num_pending = 0;
  int64_t num_redelivered = 0;
  int64_t num_dropped = 0;
};

struct Stream {
  StreamConfig cfg;
  std::deque<std::unique_ptr<Stored>> msgs;  // msgs[k] <-> seq base + k (null = dropped)
  int64_t base = 1;
  int64_t first_seq = 1;
  int64_t last_seq = 0;
  int64_t count = 0;
  int64_t bytes = 0;
  std::map<std::string, Consumer> consumers;  // ordered: deterministic snapshots

  Stored* get(int64_t seq) {
    if (seq < base || seq >= base + (int64_t)msgs.size()) return nullptr;
    return msgs[seq - base].get();
  }
  bool has(int64_t seq) { return get(seq) != nullptr; }
};

using JournalFn = std::function<void(const char* kind, mp::Value&& args)>;
// Hot-path records written straight into the journal buffer (same bytes as the
// generic JournalFn path would frame, without building an mp::Value per message)
struct JournalSink {
  virtual ~JournalSink() = default;
  virtual void store(const std::string& stream, int64_t seq, const std::string& subject, const std::string& data,
                     double ts, const mp::Value& headers) = 0;
  virtual void ack(const char* kind, const std::string& stream, const std::string& durable, int64_t seq) = 0;
};

class Engine {
 public:
  std::map<std::string, Stream> streams;  // ordered like Python's insertion for the single default stream
  std::vector<std::string> order;         // insertion order of streams (routing priority)
  JournalFn journal;                      // empty = no journal (replay)
  JournalSink* fast = nullptr;            // store / ack records (set with `journal`)
  std::function<double()> clock;

  explicit Engine(std::function<double()> clk) : clock(std::move(clk)) {}

  // ------------------------------------------------------------- helpers
  bool matches(const std::string& filt, const std::string& subject) {
    std::string key;
    key.reserve(filt.size() + subject.size() + 1);
    key.append(filt).push_back('\0');
    key.append(subject);
    auto it = match_cache_.find(key);
    if (it != match_cache_.end()) return it->second;
    bool r = subject_matches(filt, subject);
    match_cache_.emplace(std::move(key), r);
    return r;
  }

  void log(const char* kind, mp::Value&& args) {
    if (journal) journal(kind, std::move(args));
  }

  Stream& stream(const std::string& name) {
    auto it = streams.find(name);
    if (it == streams.end()) throw BusError("stream '" + name + "' not found");
    return it->second;
  }

  Consumer& consumer(const std::string& s, const std::string& d, Stream** out = nullptr) {
    Stream& st = stream(s);
    auto it = st.consumers.find(d);
    if (it == st.consumers.end()) throw BusError("consumer '" + d + "' not found on stream '" + s + "'");
    if (out) *out = &st;
    return it->second;
  }

  // ------------------------------------------------------------- streams
  void add_or_update_stream(const StreamConfig& cfg) {
    auto it = streams.find(cfg.name);
    if (it == streams.end()) {
      for (auto& nm : order) {
        Stream& other = streams[nm];
        for (auto& s : cfg.subjects)
          for (auto& o : other.cfg.subjects)
            if (subject_matches(o, s) || subject_matches(s, o))
              throw BusError("subject '" + s + "' overlaps stream '" + other.cfg.name + "'");
      }
      Stream& st = streams[cfg.name];
      st.cfg = cfg;
      order.push_back(cfg.name);
    } else {
      it->second.cfg = cfg;
    }
    route_cache_.clear();
    mp::Value a = mp::Value::arr();
    a.push(mp::Value::str(cfg.name));
    mp::Value subs = mp::Value::arr();
    for (auto& s : cfg.subjects) subs.push(mp::Value::str(s));
    a.push(std::move(subs));
    a.push(mp::Value::real(cfg.max_age));
    a.push(mp::Value::integer(cfg.max_msgs));
    a.push(mp::Value::integer(cfg.max_bytes));
    a.push(mp::Value::str(cfg.storage));
    log("stream", std::move(a));
  }

  Stream& route(const std::string& subject) {
    auto it = route_cache_.find(subject);
    if (it != route_cache_.end()) {
      if (!it->second) throw BusError("no stream matches subject '" + subject + "'");
      return *it->second;
    }
    Stream* found = nullptr;
    for (auto& nm : order) {
      Stream& cand = streams[nm];
      for (auto& p : cand.cfg.subjects)
        if (subject_matches(p, subject)) { found = &cand; break; }
      if (found) break;
    }
    route_cache_[subject] = found;
    if (!found) throw BusError("no stream matches subject '" + subject + "'");
    return *found;
  }

  // Store one message; ``seq``/``ts`` < 0 = assign.  Returns (stream, seq).
  std::pair<const std::string*, int64_t> store(const std::string& subject, std::string&& data,
                                               mp::Value&& headers, double ts = -1, int64_t seq = -1) {
    Stream& st = route(subject);
    if (ts < 0) ts = clock();
    if (seq < 0) seq = st.last_seq + 1;
    if (st.count == 0) {  // (re)anchor the window: nothing stored, seqs may jump (replay)
      st.msgs.clear();
      st.base = seq;
    } else if (seq < st.base) {
      throw BusError("sequence below the stored window");
    }
    while (st.base + (int64_t)st.msgs.size() <= seq) st.msgs.emplace_back(nullptr);
    st.last_seq = seq;
    auto m = std::make_unique<Stored>();
    m->seq = seq;
    m->subject = subject;
    m->data = std::move(data);
    m->ts = ts;
    m->headers = std::move(headers);
    st.bytes += (int64_t)m->data.size();
    st.count += 1;
    for (auto& kv : st.consumers) {
      Consumer& c = kv.second;
      if (seq > c.cursor && matches(c.cfg.filter_subject, subject)) c.num_pending += 1;
    }
    if (fast) {
      fast->store(st.cfg.name, seq, subject, m->data, ts, m->headers);
    } else if (journal) {
      mp::Value a = mp::Value::arr();
      a.push(mp::Value::str(st.cfg.name));
      a.push(mp::Value::integer(seq));
      a.push(mp::Value::str(subject));
      a.push(mp::Value::bin(m->data));
      a.push(mp::Value::real(ts));
      a.push(m->headers);
      journal("store", std::move(a));
    }
    st.msgs[seq - st.base] = std::move(m);
    enforce_limits(st);
    return {&st.cfg.name, seq};
  }

  void drop(Stream& st, int64_t seq) {
    Stored* m = st.get(seq);
    if (!m) return;
    st.bytes -= (int64_t)m->data.size();
    st.count -= 1;
    for (auto& kv : st.consumers) {
      Consumer& c = kv.second;
      if (seq > c.cursor) {
        if (matches(c.cfg.filter_subject, m->subject)) c.num_pending -= 1;
      } else {
        c.pending.erase(seq);
      }
    }
    st.msgs[seq - st.base].reset();
    trim_front(st);
  }

  void trim_front(Stream& st) {
    while (!st.msgs.empty() && !st.msgs.front()) {
      st.msgs.pop_front();
      st.base += 1;
    }
    if (st.msgs.empty()) st.base = st.last_seq + 1;
  }

  void skip_holes(Stream& st) {
    while (st.first_seq <= st.last_seq && !st.has(st.first_seq)) st.first_seq += 1;
  }

  void enforce_limits(Stream& st) {
    skip_holes(st);
    if (st.cfg.max_msgs >= 0)
      while (st.count > st.cfg.max_msgs) { drop(st, st.first_seq); st.first_seq += 1; }
    if (st.cfg.max_bytes >= 0)
      while (st.bytes > st.cfg.max_bytes && st.count > 0) { drop(st, st.first_seq); st.first_seq += 1; }
    skip_holes(st);
  }

  int64_t expire(double now) {
    int64_t n = 0;
    for (auto& nm : order) {
      Stream& st = streams[nm];
      if (st.cfg.max_age <= 0) continue;
      double horizon = now - st.cfg.max_age;
      while (st.first_seq <= st.last_seq) {
        Stored* m = st.get(st.first_seq);
        if (m) {
          if (m->ts >= horizon) break;
          drop(st, st.first_seq);
          n += 1;
        }
        st.first_seq += 1;
      }
    }
    return n;
  }

  void purge(const std::string& name) {
    Stream& st = stream(name);
    for (int64_t s = st.first_seq; s <= st.last_seq; ++s) drop(st, s);
    st.first_seq = st.last_seq + 1;
    mp::Value a = mp::Value::arr();
    a.push(mp::Value::str(name));
    log("purge", std::move(a));
  }

  // ------------------------------------------------------------- consumers
  void add_consumer(const std::string& sname, const ConsumerConfig& cfg) {
    Stream& st = stream(sname);
    auto it = st.consumers.find(cfg.durable);
    Consumer* c;
    if (it == st.consumers.end()) {
      int64_t cursor;
      if (cfg.deliver_policy == "all") {
        cursor = st.first_seq - 1;
      } else if (cfg.deliver_policy == "new") {
        cursor = st.last_seq;
      } else if (cfg.deliver_policy == "last") {
        cursor = st.last_seq;
        for (int64_t s = st.last_seq; s >= st.first_seq; --s) {
          Stored* m = st.get(s);
          if (m && subject_matches(cfg.filter_subject, m->subject)) { cursor = s - 1; break; }
        }
      } else {
        throw BusError("'" + cfg.deliver_policy + "' is not a valid DeliverPolicy");
      }
      c = &st.consumers[cfg.durable];
      c->cfg = cfg;
      c->cursor = cursor;
      recount(st, *c);
    } else {
      c = &it->second;
      ConsumerConfig old = c->cfg;
      ConsumerConfig nc = cfg;
      nc.filter_subject = old.filter_subject;
      nc.deliver_policy = old.deliver_policy;
      c->cfg = nc;
      if (cfg.filter_subject != old.filter_subject)
        throw BusError("durable '" + cfg.durable + "' is bound to '" + old.filter_subject + "', not '" +
                       cfg.filter_subject + "'");
    }
    mp::Value a = mp::Value::arr();
    a.push(mp::Value::str(sname));
    a.push(mp::Value::str(cfg.durable));
    a.push(mp::Value::str(cfg.filter_subject));
    a.push(mp::Value::real(cfg.ack_wait));
    a.push(mp::Value::integer(cfg.max_deliver));
    a.push(mp::Value::str(cfg.deliver_policy));
    a.push(mp::Value::integer(cfg.max_ack_pending));
    a.push(mp::Value::integer(c->cursor));
    log("consumer", std::move(a));
  }

  void recount(Stream& st, Consumer& c) {
    int64_t n = 0;
    for (int64_t s = std::max(c.cursor + 1, st.base); s <= st.last_seq; ++s) {
      Stored* m = st.get(s);
      if (m && matches(c.cfg.filter_subject, m->subject)) ++n;
    }
    c.num_pending = n;
  }

  void delete_stream(const std::string& name) {
    stream(name);  // throws if missing
    streams.erase(name);
    order.erase(std::remove(order.begin(), order.end(), name), order.end());
    clear_caches();
    mp::Value a = mp::Value::arr();
    a.push(mp::Value::str(name));
    log("delstream", std::move(a));
  }

  void delete_consumer(const std::string& s, const std::string& d) {
    stream(s).consumers.erase(d);
    mp::Value a = mp::Value::arr();
    a.push(mp::Value::str(s));
    a.push(mp::Value::str(d));
    log("delconsumer", std::move(a));
  }

  std::vector<Delivery> next_batch(const std::string& sname, const std::string& durable, int64_t n, double now) {
    Stream* stp;
    Consumer& c = consumer(sname, durable, &stp);
    Stream& st = *stp;
    std::vector<Delivery> out;
    // 1) redeliveries whose ack-wait (or nak delay) elapsed
    while (!c.heap.empty() && (int64_t)out.size() < n && c.heap.top().first <= now) {
      auto [ready, seq] = c.heap.top();
      c.heap.pop();
      auto it = c.pending.find(seq);
      if (it == c.pending.end() || it->second.deadline != ready) continue;  // stale
      Stored* m = st.get(seq);
      if (!m) { c.pending.erase(it); continue; }
      if (c.cfg.max_deliver > 0 && c.cfg.max_deliver <= it->second.delivered) {
        c.pending.erase(it);
        c.num_dropped += 1;
        mp::Value a = mp::Value::arr();
        a.push(mp::Value::str(sname));
        a.push(mp::Value::str(durable));
        a.push(mp::Value::integer(seq));
        log("term", std::move(a));
        continue;
      }
      it->second.delivered += 1;
      it->second.deadline = now + c.cfg.ack_wait;
      c.heap.emplace(it->second.deadline, seq);
      c.num_redelivered += 1;
      out.push_back({m, it->second.delivered});
    }
    // 2) first deliveries past the cursor
    int64_t room = c.cfg.max_ack_pending - (int64_t)c.pending.size();
    int64_t start = c.cursor;
    while ((int64_t)out.size() < n && room > 0 && c.cursor < st.last_seq) {
      c.cursor += 1;
      Stored* m = st.get(c.cursor);
      if (!m || !matches(c.cfg.filter_subject, m->subject)) continue;
      c.num_pending -= 1;
      double deadline = now + c.cfg.ack_wait;
      c.pending[m->seq] = {deadline, 1};
      c.heap.emplace(deadline, m->seq);
      out.push_back({m, 1});
      room -= 1;
    }
    if (c.cursor != start) {
      mp::Value a = mp::Value::arr();
      a.push(mp::Value::str(sname));
      a.push(mp::Value::str(durable));
      a.push(mp::Value::integer(c.cursor));
      log("cursor", std::move(a));
    }
    return out;
  }

  bool ack(const std::string& s, const std::string& d, int64_t seq, const char* kind = "ack") {
    Consumer& c = consumer(s, d);
    bool hit = c.pending.erase(seq) > 0;
    if (hit) {
      if (kind[0] == 't') c.num_dropped += 1;
      if (fast) {
        fast->ack(kind, s, d, seq);
      } else if (journal) {
        mp::Value a = mp::Value::arr();
        a.push(mp::Value::str(s));
        a.push(mp::Value::str(d));
        a.push(mp::Value::integer(seq));
        log(kind, std::move(a));
      }
    }
    return hit;
  }

  bool nak(const std::string& s, const std::string& d, int64_t seq, double delay, double now) {
    Consumer& c = consumer(s, d);
    auto it = c.pending.find(seq);
    if (it == c.pending.end()) return false;
    it->second.deadline = now + std::max(0.0, delay);
    c.heap.emplace(it->second.deadline, seq);
    return true;
  }

  bool touch(const std::string& s, const std::string& d, int64_t seq, double now) {
    Consumer& c = consumer(s, d);
    auto it = c.pending.find(seq);
    if (it == c.pending.end()) return false;
    it->second.deadline = now + c.cfg.ack_wait;
    c.heap.emplace(it->second.deadline, seq);
    return true;
  }

  // Earliest redelivery time (NAN = none); drops stale heap heads.
  double next_ready_at(Consumer& c) {
    while (!c.heap.empty()) {
      auto [ready, seq] = c.heap.top();
      auto it = c.pending.find(seq);
      if (it == c.pending.end() || it->second.deadline != ready) { c.heap.pop(); continue; }
      return ready;
    }
    return NAN;
  }

  bool has_new(Consumer& c) { return c.num_pending > 0 && (int64_t)c.pending.size() < c.cfg.max_ack_pending; }

  mp::Value consumer_info(const std::string& s, const std::string& d) {
    Consumer& c = consumer(s, d);
    int64_t floor = c.cursor;
    if (!c.pending.empty()) {
      int64_t mn = INT64_MAX;
      for (auto& kv : c.pending) mn = std::min(mn, kv.first);
      floor = mn - 1;
    }
    mp::Value v = mp::Value::map();
    v.put("stream", mp::Value::str(s));
    v.put("name", mp::Value::str(d));
    v.put("num_pending", mp::Value::integer(c.num_pending));
    v.put("num_ack_pending", mp::Value::integer((int64_t)c.pending.size()));
    v.put("num_redelivered", mp::Value::integer(c.num_redelivered));
    v.put("delivered_seq", mp::Value::integer(c.cursor));
    v.put("ack_floor", mp::Value::integer(floor));
    v.put("num_waiting", mp::Value::integer(0));
    return v;
  }

  static mp::Value config_value(const StreamConfig& c) {
    mp::Value v = mp::Value::map();
    v.put("name", mp::Value::str(c.name));
    mp::Value subs = mp::Value::arr();
    for (auto& s : c.subjects) subs.push(mp::Value::str(s));
    v.put("subjects", std::move(subs));
    v.put("max_age", mp::Value::real(c.max_age));
    v.put("max_msgs", mp::Value::integer(c.max_msgs));
    v.put("max_bytes", mp::Value::integer(c.max_bytes));
    v.put("storage", mp::Value::str(c.storage));
    return v;
  }

  mp::Value stream_info(const std::string& name) {
    Stream& st = stream(name);
    mp::Value v = mp::Value::map();
    v.put("config", config_value(st.cfg));
    v.put("messages", mp::Value::integer(st.count));
    v.put("bytes", mp::Value::integer(st.bytes));
    v.put("first_seq", mp::Value::integer(st.first_seq));
    v.put("last_seq", mp::Value::integer(st.last_seq));
    v.put("consumers", mp::Value::integer((int64_t)st.consumers.size()));
    return v;
  }

  void clear_caches() {
    route_cache_.clear();
    match_cache_.clear();
  }

 private:
  std::unordered_map<std::string, bool> match_cache_;
  std::unordered_map<std::string, Stream*> route_cache_;
};

}  // namespace bus
