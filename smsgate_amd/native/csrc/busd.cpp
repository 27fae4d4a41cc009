// smsgate-busd — native durable bus broker (the NATS-server role).
//
// Drop-in replacement for ``python -m smsgate_amd bus-server`` (bus/server.py):
// the same length-prefixed msgpack protocol (``[u32 len][msgpack]``; requests
// ``[op, req_id, *args]``, replies ``[req_id, ok, result]``, ``req_id == 0`` =
// fire-and-forget), so ``RemoteBus`` clients (bus/client.py) talk to either,
// and the same CRC-framed journal (bus/filelog.py), so either broker recovers
// the other's data directory.
//
// Design: one epoll event loop owns the engine (engine.hpp) — no locks, the
// engine is a pure state machine as in the Python broker.  Journal records
// produced while handling one batch of socket reads are group-committed with
// a single write(2) *before* any reply of that batch is sent, so an
// acknowledged publish is in the OS page cache (and, with --fsync always, on
// disk).  Long-poll fetches park as waiters; after every loop iteration the
// waiters are retried (publishes, naks, acks and redelivery deadlines can all
// make messages available) and the epoll timeout is the earliest waiter
// deadline / redelivery time / 1 s retention tick.  With ``--fsync interval``
// (the default) the periodic fdatasync runs on a background thread, so the event
// loop only ever pays for the write(2) into the page cache; ``--fsync always``
// keeps the sync inline before the replies of the batch.
//
// Usage: smsgate-busd --listen tcp://0.0.0.0:4222 [--listen unix:///run/bus.sock]
//                     [--data DIR] [--max-age S] [--fsync interval|always|never]
//                     [--fsync-interval S] [--compact-bytes N]
// ``--nats-listen tcp://HOST:PORT`` adds the NATS client protocol + JetStream API
// front-end (Server::nats_*) on the same engine.
// Prints ``READY <tcp-port|->[ NATS <port>]`` on stdout once listening.
#include <arpa/inet.h>
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/un.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine.hpp"
#include "http_ingest.hpp"
#include "json.hpp"

namespace {

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

double wall_now() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return tv.tv_sec + tv.tv_usec * 1e-6;
}

double mono_now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

[[noreturn]] void die(const std::string& msg) {
  fprintf(stderr, "smsgate-busd: %s\n", msg.c_str());
  exit(2);
}

bool write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = ::write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

void put_u32(std::string& o, uint32_t v) {
  char b[4] = {(char)(v & 0xff), (char)((v >> 8) & 0xff), (char)((v >> 16) & 0xff), (char)(v >> 24)};
  o.append(b, 4);
}

uint32_t get_u32(const char* p) {
  const uint8_t* u = (const uint8_t*)p;
  return u[0] | (u[1] << 8) | (u[2] << 16) | ((uint32_t)u[3] << 24);
}

// ------------------------------------------------------------------- journal
class Journal : public bus::JournalSink {
 public:
  Journal(std::string dir, std::string mode, double interval, int64_t compact_bytes)
      : dir_(std::move(dir)), mode_(std::move(mode)), interval_(interval), compact_bytes_(compact_bytes) {
    if (mode_ == "interval") syncer_ = std::thread([this] { sync_loop(); });
  }

  ~Journal() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (syncer_.joinable()) syncer_.join();
  }

  std::vector<std::string> segments() const {
    std::vector<std::string> out;
    DIR* d = opendir(dir_.c_str());
    if (!d) return out;
    while (dirent* e = readdir(d)) {
      std::string n = e->d_name;
      if (n.size() == 20 && n.rfind("journal-", 0) == 0 && n.substr(16) == ".log") out.push_back(n);
    }
    closedir(d);
    std::sort(out.begin(), out.end());
    return out;
  }

  std::string path(int n) const {
    char b[32];
    snprintf(b, sizeof b, "journal-%08d.log", n);
    return dir_ + "/" + b;
  }

  void open_segment(int n) {
    if (fd_ >= 0) {
      flush();
      std::lock_guard<std::mutex> g(mu_);  // not while the syncer holds the old fd
      ::fsync(fd_);
      ::close(fd_);
      sync_fd_ = -1;
    }
    seg_ = n;
    fd_ = ::open(path(n).c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (fd_ < 0) die("cannot open journal segment " + path(n));
    {
      std::lock_guard<std::mutex> g(mu_);
      sync_fd_ = fd_;
    }
    struct stat sb;
    fstat(fd_, &sb);
    bytes_ = sb.st_size;
    floor_bytes_ = bytes_;  // a fresh segment is a snapshot (compaction) or the recovered tail
  }

  static void frame(std::string& out, const char* kind, const mp::Value& args) {
    std::string body;
    body.reserve(64 + args.a.size() * 16);
    mp::enc_arr_hdr(body, 2);
    mp::enc_str(body, kind, strlen(kind));
    mp::encode(body, args);
    put_u32(out, (uint32_t)body.size());
    put_u32(out, crc::crc32(body.data(), body.size()));
    out += body;
  }

  void append(const char* kind, mp::Value&& args) {
    size_t before = buf_.size();
    frame(buf_, kind, args);
    bytes_ += (int64_t)(buf_.size() - before);
    // compact only once the journal has doubled since the last snapshot: when the live
    // state itself exceeds compact_bytes, a fixed threshold would re-compact after
    // every append (the whole state rewritten on the event loop, over and over)
    if (bytes_ > std::max(compact_bytes_, 2 * floor_bytes_)) need_compact = true;
  }

  // Hot-path records encoded in place: [len][crc][ ["store", [stream, seq, subject,
  // bin(data), ts, headers]] ] -- the bytes frame() produces for the same record.
  void store(const std::string& stream, int64_t seq, const std::string& subject, const std::string& data, double ts,
             const mp::Value& headers) override {
    const size_t at = begin_record();
    mp::enc_arr_hdr(buf_, 2);
    mp::enc_str(buf_, "store", 5);
    mp::enc_arr_hdr(buf_, 6);
    mp::enc_str(buf_, stream);
    mp::enc_int(buf_, seq);
    mp::enc_str(buf_, subject);
    mp::enc_bin(buf_, data.data(), data.size());
    mp::enc_double(buf_, ts);
    mp::encode(buf_, headers);
    end_record(at);
  }

  void ack(const char* kind, const std::string& stream, const std::string& durable, int64_t seq) override {
    const size_t at = begin_record();
    mp::enc_arr_hdr(buf_, 2);
    mp::enc_str(buf_, kind, strlen(kind));
    mp::enc_arr_hdr(buf_, 3);
    mp::enc_str(buf_, stream);
    mp::enc_str(buf_, durable);
    mp::enc_int(buf_, seq);
    end_record(at);
  }

  // Group commit: one write(2) for everything appended since the last flush.
  void flush() {
    if (buf_.empty() || fd_ < 0) return;
    if (!write_all(fd_, buf_.data(), buf_.size())) die("journal write failed");
    buf_.clear();
    dirty_ = true;
    if (mode_ == "always") sync();
    else if (mode_ == "interval" && mono_now() - last_sync_ >= interval_) sync();
  }

  void sync() {
    if (fd_ >= 0 && dirty_) {
      if (syncer_.joinable()) {  // interval mode: hand the fdatasync to the syncer thread
        {
          std::lock_guard<std::mutex> g(mu_);
          want_sync_ = true;
        }
        cv_.notify_one();
      } else {
        ::fdatasync(fd_);
      }
    }
    dirty_ = false;
    last_sync_ = mono_now();
  }

  // Seconds until an interval fsync is due (large if nothing is dirty).
  double sync_due_in() const {
    if (mode_ != "interval" || !dirty_) return 1e9;
    return std::max(0.0, interval_ - (mono_now() - last_sync_));
  }

  void tick() {
    if (mode_ == "interval" && dirty_ && mono_now() - last_sync_ >= interval_) sync();
  }

  void close() {
    if (fd_ >= 0) {
      flush();
      std::lock_guard<std::mutex> g(mu_);
      ::fsync(fd_);
      ::close(fd_);
      fd_ = -1;
      sync_fd_ = -1;
    }
  }

  int seg() const { return seg_; }
  const std::string& dir() const { return dir_; }

  bool need_compact = false;

 private:
  std::string dir_, mode_;
  double interval_;
  int64_t compact_bytes_;
  int fd_ = -1;
  int seg_ = 0;
  int64_t bytes_ = 0;
  int64_t floor_bytes_ = 0;  // journal size right after the last snapshot
  std::string buf_;
  bool dirty_ = false;
  double last_sync_ = 0.0;
  // background fdatasync (interval mode); mu_ guards sync_fd_ against segment rotation
  std::thread syncer_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool want_sync_ = false, stop_ = false;
  int sync_fd_ = -1;

  size_t begin_record() {
    const size_t at = buf_.size();
    buf_.append(8, '\0');  // length + CRC, patched by end_record
    return at;
  }

  void end_record(size_t at) {
    const size_t n = buf_.size() - at - 8;
    const uint32_t c = crc::crc32(buf_.data() + at + 8, n);
    for (int k = 0; k < 4; ++k) {
      buf_[at + k] = (char)((n >> (8 * k)) & 0xff);
      buf_[at + 4 + k] = (char)((c >> (8 * k)) & 0xff);
    }
    bytes_ += (int64_t)(n + 8);
    if (bytes_ > std::max(compact_bytes_, 2 * floor_bytes_)) need_compact = true;
  }

  void sync_loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return want_sync_ || stop_; });
      if (stop_) return;
      want_sync_ = false;
      if (sync_fd_ >= 0) ::fdatasync(sync_fd_);  // under mu_: the fd cannot be closed meanwhile
    }
  }
};

// ------------------------------------------------------------- replay (recovery)
bus::ConsumerConfig consumer_cfg(const std::vector<mp::Value>& a, size_t off) {
  bus::ConsumerConfig c;
  c.durable = a[off].as_str();
  c.filter_subject = a[off + 1].as_str();
  c.ack_wait = a[off + 2].as_double();
  c.max_deliver = a[off + 3].as_int();
  c.deliver_policy = a[off + 4].as_str();
  c.max_ack_pending = a[off + 5].as_int();
  return c;
}

bus::StreamConfig stream_cfg_from_args(const std::vector<mp::Value>& a) {
  bus::StreamConfig c;
  c.name = a[0].as_str();
  for (auto& s : a[1].as_arr()) c.subjects.push_back(s.as_str());
  c.max_age = a[2].as_double();
  c.max_msgs = a[3].as_int();
  c.max_bytes = a[4].as_int();
  c.storage = a[5].is_nil() ? "file" : a[5].as_str();
  return c;
}

// Mirrors filelog.replay_into (bus/filelog.py:55-108).
void replay_into(bus::Engine& eng, const std::string& kind, mp::Value& args) {
  auto& a = args.a;
  if (kind == "stream") {
    eng.add_or_update_stream(stream_cfg_from_args(a));
  } else if (kind == "store") {
    bus::Stream& st = eng.stream(a[0].as_str());
    int64_t seq = a[1].as_int();
    if (seq > st.last_seq) {
      std::string data = a[3].s;
      eng.store(a[2].as_str(), std::move(data), std::move(a[5]), a[4].as_double(), seq);
    }
  } else if (kind == "consumer") {
    bus::Stream& st = eng.stream(a[0].as_str());
    bus::ConsumerConfig cfg = consumer_cfg(a, 1);
    int64_t cursor = a[7].as_int();
    auto it = st.consumers.find(cfg.durable);
    if (it == st.consumers.end()) {
      eng.add_consumer(st.cfg.name, cfg);
      bus::Consumer& c = st.consumers[cfg.durable];
      c.cursor = cursor;
      eng.recount(st, c);
    } else {
      it->second.cfg = cfg;
    }
  } else if (kind == "cursor") {
    bus::Stream& st = eng.stream(a[0].as_str());
    auto it = st.consumers.find(a[1].as_str());
    if (it == st.consumers.end()) return;
    bus::Consumer& c = it->second;
    int64_t nw = a[2].as_int();
    for (int64_t s = c.cursor + 1; s <= nw; ++s) {
      bus::Stored* m = st.get(s);
      if (m && eng.matches(c.cfg.filter_subject, m->subject)) {
        c.pending[s] = {0.0, 1};  // delivered before the crash: redeliver at once
        c.num_pending -= 1;
      }
    }
    c.cursor = std::max(c.cursor, nw);
  } else if (kind == "ack" || kind == "term") {
    bus::Stream& st = eng.stream(a[0].as_str());
    auto it = st.consumers.find(a[1].as_str());
    if (it != st.consumers.end()) it->second.pending.erase(a[2].as_int());
  } else if (kind == "delstream") {
    if (eng.streams.count(a[0].as_str())) eng.delete_stream(a[0].as_str());
  } else if (kind == "delconsumer") {
    eng.stream(a[0].as_str()).consumers.erase(a[1].as_str());
  } else if (kind == "purge") {
    eng.purge(a[0].as_str());
  } else if (kind == "pending") {
    bus::Stream& st = eng.stream(a[0].as_str());
    auto it = st.consumers.find(a[1].as_str());
    if (it == st.consumers.end()) return;
    for (auto& s : a[2].as_arr()) {
      int64_t q = s.as_int();
      if (st.has(q)) it->second.pending[q] = {0.0, 1};
    }
  }
}

void recover(bus::Engine& eng, Journal& jr) {
  mkdir(jr.dir().c_str(), 0755);
  auto segs = jr.segments();
  for (auto& name : segs) {
    std::string p = jr.dir() + "/" + name;
    FILE* f = fopen(p.c_str(), "rb");
    if (!f) die("cannot read " + p);
    std::string data;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) data.append(buf, n);
    fclose(f);
    size_t off = 0, good = 0;
    while (off + 8 <= data.size()) {
      uint32_t len = get_u32(data.data() + off), c = get_u32(data.data() + off + 4);
      size_t end = off + 8 + len;
      if (end > data.size()) break;
      if (crc::crc32(data.data() + off + 8, len) != c) break;
      mp::Value rec;
      try {
        rec = mp::decode(data.data() + off + 8, len);
      } catch (std::exception&) {
        break;
      }
      if (rec.t == mp::Value::ARR && rec.a.size() == 2 && rec.a[0].t == mp::Value::STR)
        replay_into(eng, rec.a[0].s, rec.a[1]);
      good = end;
      off = end;
    }
    if (good != data.size()) {  // torn tail: drop it
      if (truncate(p.c_str(), (off_t)good) != 0) die("cannot truncate torn journal tail of " + p);
    }
  }
  for (auto& nm : eng.order) {
    bus::Stream& st = eng.streams[nm];
    for (auto& kv : st.consumers) {
      bus::Consumer& c = kv.second;
      eng.recount(st, c);
      for (auto& pv : c.pending) c.heap.emplace(pv.second.deadline, pv.first);  // redeliver unacked at once
    }
  }
  int last = 1;
  if (!segs.empty()) last = atoi(segs.back().c_str() + 8);
  jr.open_segment(last);
}

// Rewrite the whole state as one fresh segment, then drop older ones (filelog.compact).
void compact(bus::Engine& eng, Journal& jr) {
  auto old = jr.segments();
  int n = jr.seg() + 1;
  std::string fin = jr.path(n), tmp = fin + ".tmp";
  std::string out;
  for (auto& nm : eng.order) {
    bus::Stream& st = eng.streams[nm];
    mp::Value a = mp::Value::arr();
    a.push(mp::Value::str(st.cfg.name));
    mp::Value subs = mp::Value::arr();
    for (auto& s : st.cfg.subjects) subs.push(mp::Value::str(s));
    a.push(std::move(subs));
    a.push(mp::Value::real(st.cfg.max_age));
    a.push(mp::Value::integer(st.cfg.max_msgs));
    a.push(mp::Value::integer(st.cfg.max_bytes));
    a.push(mp::Value::str(st.cfg.storage));
    Journal::frame(out, "stream", a);
    for (int64_t s = st.first_seq; s <= st.last_seq; ++s) {
      bus::Stored* m = st.get(s);
      if (!m) continue;
      mp::Value r = mp::Value::arr();
      r.push(mp::Value::str(st.cfg.name));
      r.push(mp::Value::integer(m->seq));
      r.push(mp::Value::str(m->subject));
      r.push(mp::Value::bin(m->data));
      r.push(mp::Value::real(m->ts));
      r.push(m->headers);
      Journal::frame(out, "store", r);
    }
    for (auto& kv : st.consumers) {
      bus::Consumer& c = kv.second;
      mp::Value r = mp::Value::arr();
      r.push(mp::Value::str(st.cfg.name));
      r.push(mp::Value::str(kv.first));
      r.push(mp::Value::str(c.cfg.filter_subject));
      r.push(mp::Value::real(c.cfg.ack_wait));
      r.push(mp::Value::integer(c.cfg.max_deliver));
      r.push(mp::Value::str(c.cfg.deliver_policy));
      r.push(mp::Value::integer(c.cfg.max_ack_pending));
      r.push(mp::Value::integer(c.cursor));
      Journal::frame(out, "consumer", r);
      std::vector<int64_t> seqs;
      for (auto& pv : c.pending) seqs.push_back(pv.first);
      std::sort(seqs.begin(), seqs.end());
      mp::Value p = mp::Value::arr();
      p.push(mp::Value::str(st.cfg.name));
      p.push(mp::Value::str(kv.first));
      mp::Value l = mp::Value::arr();
      for (auto q : seqs) l.push(mp::Value::integer(q));
      p.push(std::move(l));
      Journal::frame(out, "pending", p);
    }
  }
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0 || !write_all(fd, out.data(), out.size())) die("compaction write failed");
  ::fsync(fd);
  ::close(fd);
  jr.flush();
  if (rename(tmp.c_str(), fin.c_str()) != 0) die("compaction rename failed");
  jr.open_segment(n);
  for (auto& s : old) {
    std::string p = jr.dir() + "/" + s;
    if (p != fin) unlink(p.c_str());
  }
}

// -------------------------------------------------------------------- server
struct NSub {  // a NATS-protocol subscription
  std::string subject, queue;
};

struct Conn {
  int fd;
  uint64_t id;
  bool nats = false;                               // NATS text protocol (--nats-listen)
  bool http = false;                               // HTTP/1.1 ingestion (--http-listen)
  bool close_after = false;                        // HTTP: close once the reply is written
  std::unordered_map<std::string, NSub> subs;      // NATS: sid -> subscription
  std::string in;
  size_t in_off = 0;
  std::string out;
  size_t out_off = 0;
  bool writing = false;
  bool dead = false;
};

// a NATS pull request ($JS.API.CONSUMER.MSG.NEXT) still being filled
struct NWaiter {
  std::string reply, stream, durable;
  int64_t batch, sent = 0;
  double deadline;
  bool no_wait;
};

struct Waiter {
  uint64_t conn;
  int64_t rid;
  std::string stream, durable;
  int64_t batch;
  double deadline;  // wall clock; INFINITY = wait forever
};

const char* kAllSubjects[] = {"sms.raw",        "sms.parsed",      "sms.failed",
                              "sms.processing", "sms.categorized", "sms.failed.final"};

class Server {
 public:
  Server(bus::Engine& eng, Journal* jr, double max_age) : eng_(eng), jr_(jr), max_age_(max_age) {
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    if (ep_ < 0) die("epoll_create1 failed");
  }

  bus::StreamConfig default_config() const {
    bus::StreamConfig c;
    c.name = "SMS";
    for (auto s : kAllSubjects) c.subjects.push_back(s);
    c.max_age = max_age_;
    return c;
  }

  int listen_on(const std::string& url, bool nats = false, bool http = false) {
    int fd;
    int port = -1;
    if (url.rfind("unix://", 0) == 0) {
      std::string path = url.substr(7);
      unlink(path.c_str());
      fd = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      sockaddr_un sa{};
      sa.sun_family = AF_UNIX;
      if (path.size() >= sizeof(sa.sun_path)) die("unix socket path too long: " + path);
      strncpy(sa.sun_path, path.c_str(), sizeof(sa.sun_path) - 1);
      if (bind(fd, (sockaddr*)&sa, sizeof sa) != 0) die("bind " + url + ": " + strerror(errno));
    } else {
      std::string hp = url.rfind("tcp://", 0) == 0 ? url.substr(6) : url;
      size_t colon = hp.rfind(':');
      std::string host = colon == std::string::npos ? hp : hp.substr(0, colon);
      std::string ps = colon == std::string::npos ? "4222" : hp.substr(colon + 1);
      if (host.empty()) host = "0.0.0.0";
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      hints.ai_flags = AI_PASSIVE;
      if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res) die("cannot resolve " + url);
      fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      int one = 1;
      setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
      if (bind(fd, res->ai_addr, res->ai_addrlen) != 0) die("bind " + url + ": " + strerror(errno));
      freeaddrinfo(res);
      sockaddr_in sa{};
      socklen_t sl = sizeof sa;
      getsockname(fd, (sockaddr*)&sa, &sl);
      port = ntohs(sa.sin_port);
    }
    if (listen(fd, 512) != 0) die("listen " + url);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.u64 = 0;  // 0 = a listener; look up by fd
    listeners_.push_back(fd);
    ev.data.u64 = (uint64_t)fd | (1ull << 63) | (nats ? (1ull << 62) : 0) | (http ? (1ull << 61) : 0);
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    return port;
  }

  void run() {
    std::vector<epoll_event> evs(256);
    last_expire_ = wall_now();
    while (!g_stop) {
      int timeout = compute_timeout_ms();
      int n = epoll_wait(ep_, evs.data(), (int)evs.size(), timeout);
      if (n < 0 && errno != EINTR) die("epoll_wait failed");
      for (int k = 0; k < n; ++k) {
        uint64_t tag = evs[k].data.u64;
        if (tag & (1ull << 63)) {
          accept_all((int)(tag & 0xffffffff), (tag >> 62) & 1, (tag >> 61) & 1);
          continue;
        }
        auto it = conns_.find(tag);
        if (it == conns_.end()) continue;
        Conn& c = it->second;
        if (evs[k].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) read_conn(c);
        // EPOLLOUT: nothing to do here -- flush_conns retries every pending write each
        // iteration; `writing` means EPOLLOUT interest is armed until the output drains
      }
      double now = wall_now();
      if (now - last_expire_ >= 1.0) {
        eng_.expire(now);
        last_expire_ = now;
      }
      serve_waiters(now);
      serve_nats(now);
      if (jr_) {
        jr_->flush();  // group commit before any reply of this iteration leaves
        jr_->tick();
        if (jr_->need_compact) {
          jr_->need_compact = false;
          compact(eng_, *jr_);
        }
      }
      flush_conns();
    }
    if (jr_) jr_->close();
  }

 private:
  int compute_timeout_ms() {
    double now = wall_now();
    double t = std::max(0.0, 1.0 - (now - last_expire_));
    for (auto& w : waiters_) {
      if (w.deadline < INFINITY) t = std::min(t, std::max(0.0, w.deadline - now));
      try {
        bus::Consumer& c = eng_.consumer(w.stream, w.durable);
        double r = eng_.next_ready_at(c);
        if (!std::isnan(r)) t = std::min(t, std::max(0.0, r - now) + 1e-4);
      } catch (std::exception&) {
        t = 0;
      }
    }
    for (auto& w : nwaiters_) {
      t = std::min(t, std::max(0.0, w.deadline - now));
      try {
        double r = eng_.next_ready_at(eng_.consumer(w.stream, w.durable));
        if (!std::isnan(r)) t = std::min(t, std::max(0.0, r - now) + 1e-4);
      } catch (std::exception&) {
        t = 0;
      }
    }
    for (auto& kv : push_) {
      try {
        double r = eng_.next_ready_at(eng_.consumer(kv.first.first, kv.first.second));
        if (!std::isnan(r)) t = std::min(t, std::max(0.0, r - now) + 1e-4);
      } catch (std::exception&) {
        t = 0;
      }
    }
    if (!push_.empty()) t = std::min(t, 0.05);  // a deliver-subject subscriber may have appeared
    if (jr_) t = std::min(t, jr_->sync_due_in());
    return (int)std::ceil(t * 1000.0);
  }

  void accept_all(int lfd, bool nats, bool http = false) {
    for (;;) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);  // harmless failure on AF_UNIX
      uint64_t id = ++next_id_;
      Conn& c = conns_[id];
      c.fd = fd;
      c.id = id;
      c.nats = nats;
      c.http = http;
      if (nats) nats_info(c);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = id;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    }
  }

  void read_conn(Conn& c) {
    char buf[1 << 16];
    for (;;) {
      ssize_t r = ::read(c.fd, buf, sizeof buf);
      if (r > 0) {
        c.in.append(buf, (size_t)r);
        continue;
      }
      if (r == 0 || (errno != EAGAIN && errno != EINTR)) c.dead = true;
      if (r < 0 && errno == EINTR) continue;
      break;
    }
    if (c.nats) nats_parse(c);
    if (c.http) http_parse(c);
    while (!c.nats && !c.http && c.in.size() - c.in_off >= 4) {
      uint32_t len = get_u32(c.in.data() + c.in_off);
      if (len > (256u << 20)) { c.dead = true; break; }
      if (c.in.size() - c.in_off < 4 + (size_t)len) break;
      mp::Value req;
      bool ok = true;
      try {
        req = mp::decode(c.in.data() + c.in_off + 4, len);
      } catch (std::exception&) {
        ok = false;
      }
      c.in_off += 4 + len;
      if (!ok || req.t != mp::Value::ARR || req.a.size() < 2) { c.dead = true; break; }
      dispatch(c, req);
    }
    if (c.in_off > 0 && c.in_off * 2 >= c.in.size()) {
      c.in.erase(0, c.in_off);
      c.in_off = 0;
    }
  }

  void reply(Conn& c, int64_t rid, bool ok, const mp::Value& res) {
    if (rid == 0) return;
    std::string body;
    mp::enc_arr_hdr(body, 3);
    mp::enc_int(body, rid);
    mp::enc_bool(body, ok);
    mp::encode(body, res);
    put_u32(c.out, (uint32_t)body.size());
    c.out += body;
  }

  void reply_raw(Conn& c, int64_t rid, const std::string& encoded_result) {
    if (rid == 0) return;
    std::string body;
    mp::enc_arr_hdr(body, 3);
    mp::enc_int(body, rid);
    mp::enc_bool(body, true);
    body += encoded_result;
    put_u32(c.out, (uint32_t)body.size());
    c.out += body;
  }

  static void encode_deliveries(std::string& o, const std::vector<bus::Delivery>& got) {
    mp::enc_arr_hdr(o, got.size());
    for (auto& d : got) {
      mp::enc_arr_hdr(o, 6);
      mp::enc_str(o, d.msg->subject);
      mp::enc_bin(o, d.msg->data.data(), d.msg->data.size());
      mp::enc_int(o, d.msg->seq);
      mp::enc_int(o, d.num_delivered);
      mp::enc_double(o, d.msg->ts);
      if (d.msg->headers.t == mp::Value::MAP && !d.msg->headers.m.empty()) mp::encode(o, d.msg->headers);
      else mp::enc_nil(o);
    }
  }

  void dispatch(Conn& c, mp::Value& req) {
    int64_t rid = 0;
    std::string op;
    try {
      op = req.a[0].as_str();
      rid = req.a[1].as_int();
      auto& a = req.a;
      const size_t A = 2;  // first argument index
      auto arg = [&](size_t k) -> mp::Value& {
        if (A + k >= a.size()) throw bus::BusError("missing argument for '" + op + "'");
        return a[A + k];
      };
      double now = wall_now();
      if (op == "ping") {
        reply(c, rid, true, mp::Value::boolean(true));
      } else if (op == "publish") {
        mp::Value hdr = a.size() > A + 2 ? std::move(a[A + 2]) : mp::Value::nil();
        std::string data = std::move(arg(1).s);
        auto r = eng_.store(arg(0).as_str(), std::move(data), std::move(hdr));
        mp::Value res = mp::Value::arr();
        res.push(mp::Value::str(*r.first));
        res.push(mp::Value::integer(r.second));
        reply(c, rid, true, res);
      } else if (op == "publish_many") {
        auto& items = arg(0).a;
        std::string o;
        mp::enc_arr_hdr(o, items.size());
        for (auto& it : items) {
          auto& pair = it.as_arr();
          if (pair.size() < 2) throw bus::BusError("publish_many item needs [subject, data]");
          std::string data = std::move(const_cast<mp::Value&>(pair[1]).s);
          auto r = eng_.store(pair[0].as_str(), std::move(data), mp::Value::nil());
          mp::enc_arr_hdr(o, 2);
          mp::enc_str(o, *r.first);
          mp::enc_int(o, r.second);
        }
        reply_raw(c, rid, o);
      } else if (op == "ensure_stream") {
        bus::StreamConfig cfg = default_config();
        if (a.size() > A && a[A].t == mp::Value::MAP) {
          const mp::Value& m = a[A];
          if (auto v = m.get("name")) cfg.name = v->as_str();
          if (auto v = m.get("subjects")) {
            cfg.subjects.clear();
            for (auto& s : v->as_arr()) cfg.subjects.push_back(s.as_str());
          }
          if (auto v = m.get("max_age")) cfg.max_age = v->as_double();
          if (auto v = m.get("max_msgs")) cfg.max_msgs = v->as_int();
          if (auto v = m.get("max_bytes")) cfg.max_bytes = v->as_int();
          if (auto v = m.get("storage")) cfg.storage = v->as_str();
        }
        auto it = eng_.streams.find(cfg.name);
        bool same = false;
        if (it != eng_.streams.end()) {
          auto x = it->second.cfg.subjects, y = cfg.subjects;
          std::sort(x.begin(), x.end());
          std::sort(y.begin(), y.end());
          same = x == y;
        }
        if (!same) eng_.add_or_update_stream(cfg);
        mp::Value res = mp::Value::map();
        res.put("name", mp::Value::str(cfg.name));
        res.put("messages", mp::Value::integer(eng_.stream(cfg.name).count));
        reply(c, rid, true, res);
      } else if (op == "subscribe") {
        const std::string& subject = arg(0).as_str();
        bus::ConsumerConfig cfg;
        cfg.durable = arg(1).as_str();
        cfg.filter_subject = subject;
        const mp::Value& opts = arg(2);
        if (opts.t == mp::Value::MAP) {
          for (auto& kv : opts.m) {
            const std::string& k = kv.first.as_str();
            if (k == "ack_wait") cfg.ack_wait = kv.second.as_double();
            else if (k == "max_deliver") cfg.max_deliver = kv.second.as_int();
            else if (k == "deliver_policy") cfg.deliver_policy = kv.second.as_str();
            else if (k == "max_ack_pending") cfg.max_ack_pending = kv.second.as_int();
            else throw bus::BusError("unexpected consumer option '" + k + "'");
          }
        }
        std::string sname = eng_.route(subject).cfg.name;
        eng_.add_consumer(sname, cfg);
        reply(c, rid, true, mp::Value::str(sname));
      } else if (op == "fetch") {
        Waiter w;
        w.conn = c.id;
        w.rid = rid;
        w.stream = arg(0).as_str();
        w.durable = arg(1).as_str();
        w.batch = std::max<int64_t>(1, arg(2).as_int());
        const mp::Value& to = arg(3);
        w.deadline = to.is_nil() ? INFINITY : now + to.as_double();
        auto got = eng_.next_batch(w.stream, w.durable, w.batch, now);
        if (!got.empty() || (!to.is_nil() && to.as_double() <= 0)) {
          std::string o;
          encode_deliveries(o, got);
          reply_raw(c, rid, o);
        } else {
          waiters_.push_back(std::move(w));
        }
      } else if (op == "ack" || op == "term") {
        eng_.ack(arg(0).as_str(), arg(1).as_str(), arg(2).as_int(), op == "ack" ? "ack" : "term");
        reply(c, rid, true, mp::Value::nil());
      } else if (op == "ack_many") {
        const std::string& s = arg(0).as_str();
        const std::string& d = arg(1).as_str();
        for (auto& q : arg(2).as_arr()) eng_.ack(s, d, q.as_int());
        reply(c, rid, true, mp::Value::nil());
      } else if (op == "nak") {
        eng_.nak(arg(0).as_str(), arg(1).as_str(), arg(2).as_int(), arg(3).as_double(), now);
        reply(c, rid, true, mp::Value::nil());
      } else if (op == "touch") {
        eng_.touch(arg(0).as_str(), arg(1).as_str(), arg(2).as_int(), now);
        reply(c, rid, true, mp::Value::nil());
      } else if (op == "consumer_info") {
        reply(c, rid, true, eng_.consumer_info(arg(0).as_str(), arg(1).as_str()));
      } else if (op == "stream_info") {
        reply(c, rid, true, eng_.stream_info(arg(0).as_str()));
      } else {
        throw bus::BusError("unknown op '" + op + "'");
      }
    } catch (bus::BusError& e) {
      reply(c, rid, false, mp::Value::str(std::string("BusError: ") + e.what()));
    } catch (std::exception& e) {
      reply(c, rid, false, mp::Value::str(std::string("ValueError: ") + e.what()));
    }
  }

  void serve_waiters(double now) {
    for (auto it = waiters_.begin(); it != waiters_.end();) {
      auto cit = conns_.find(it->conn);
      if (cit == conns_.end() || cit->second.dead) {
        it = waiters_.erase(it);
        continue;
      }
      std::vector<bus::Delivery> got;
      bool fail = false;
      std::string err;
      try {
        got = eng_.next_batch(it->stream, it->durable, it->batch, now);
      } catch (std::exception& e) {
        fail = true;
        err = std::string("BusError: ") + e.what();
      }
      if (fail) {
        reply(cit->second, it->rid, false, mp::Value::str(err));
        it = waiters_.erase(it);
      } else if (!got.empty() || now >= it->deadline) {
        std::string o;
        encode_deliveries(o, got);
        reply_raw(cit->second, it->rid, o);
        it = waiters_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void flush_conns() {
    for (auto it = conns_.begin(); it != conns_.end();) {
      Conn& c = it->second;
      while (!c.dead && c.out_off < c.out.size()) {
        ssize_t w = ::write(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off);
        if (w > 0) {
          c.out_off += (size_t)w;
        } else if (w < 0 && errno == EINTR) {
          continue;
        } else if (w < 0 && errno == EAGAIN) {
          if (!c.writing) {
            epoll_event ev{};
            ev.events = EPOLLIN | EPOLLRDHUP | EPOLLOUT;
            ev.data.u64 = c.id;
            epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &ev);
            c.writing = true;
          }
          break;
        } else {
          c.dead = true;
        }
      }
      if (c.close_after && c.out_off == c.out.size()) c.dead = true;  // HTTP "Connection: close": reply sent
      if (c.out_off == c.out.size() && !c.out.empty()) {
        c.out.clear();
        c.out_off = 0;
        if (c.writing) {  // EPOLLOUT was armed by a short write: back to read-only interest
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.u64 = c.id;
          epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &ev);
          c.writing = false;
        }
      }
      if (c.dead) {
        epoll_ctl(ep_, EPOLL_CTL_DEL, c.fd, nullptr);
        ::close(c.fd);
        it = conns_.erase(it);
      } else {
        ++it;
      }
    }
  }


  // =================================================================== HTTP
  // Native ingestion front-end (``--http-listen``): the gateway's POST /sms/raw and
  // POST /sms/raw/batch contract (http_ingest.hpp) plus GET /health and GET
  // /metrics, HTTP/1.1 keep-alive (pipelined requests are answered in order).  An
  // accepted SMS is stored on sms.raw by this loop's engine and its journal record
  // is group-committed before the 202 leaves, like a msgpack publish.
  static constexpr size_t kHttpMaxHeader = 64u << 10, kHttpMaxBody = 64u << 20;

  static std::string lower(std::string s) {
    for (auto& ch : s) ch = (char)tolower((unsigned char)ch);
    return s;
  }

  void http_reply(Conn& c, int status, const std::string& body, bool keep_alive,
                  const char* ctype = "application/json") {
    const char* reason = status == 200   ? "OK"
                         : status == 202 ? "Accepted"
                         : status == 400 ? "Bad Request"
                         : status == 404 ? "Not Found"
                         : status == 405 ? "Method Not Allowed"
                         : status == 413 ? "Content Too Large"
                         : status == 422 ? "Unprocessable Entity"
                         : status == 431 ? "Request Header Fields Too Large"
                         : status == 501 ? "Not Implemented"
                                         : "Internal Server Error";
    c.out += "HTTP/1.1 " + std::to_string(status) + " " + reason + "\r\ncontent-length: " +
             std::to_string(body.size()) + "\r\ncontent-type: " + ctype + "\r\n" +
             (keep_alive ? "" : "connection: close\r\n") + "\r\n" + body;
    if (!keep_alive) c.close_after = true;
  }

  void http_parse(Conn& c) {
    while (!c.dead && !c.close_after) {
      const char* base = c.in.data() + c.in_off;
      const size_t avail = c.in.size() - c.in_off;
      const char* he = (const char*)memmem(base, avail, "\r\n\r\n", 4);
      if (!he) {
        if (avail > kHttpMaxHeader) http_reply(c, 431, "{\"detail\":\"Request Header Fields Too Large\"}", false);
        return;
      }
      const size_t hlen = (size_t)(he - base) + 4;
      const std::string head(base, hlen - 4);
      const size_t eol = head.find("\r\n");
      const std::string line = head.substr(0, eol);
      const size_t sp1 = line.find(' '), sp2 = line.rfind(' ');
      if (sp1 == std::string::npos || sp2 == sp1) {
        http_reply(c, 400, "{\"detail\":\"Bad Request\"}", false);
        return;
      }
      const std::string method = line.substr(0, sp1), version = line.substr(sp2 + 1);
      std::string path = line.substr(sp1 + 1, sp2 - sp1 - 1);
      bool keep_alive = version == "HTTP/1.1";
      long long clen = 0;
      bool chunked = false;
      size_t pos = eol == std::string::npos ? head.size() : eol + 2;
      while (pos < head.size()) {
        size_t e = head.find("\r\n", pos);
        if (e == std::string::npos) e = head.size();
        const std::string h = head.substr(pos, e - pos);
        pos = e + 2;
        const size_t colon = h.find(':');
        if (colon == std::string::npos) continue;
        const std::string name = lower(h.substr(0, colon));
        size_t v0 = colon + 1;
        while (v0 < h.size() && (h[v0] == ' ' || h[v0] == '\t')) ++v0;
        const std::string val = lower(h.substr(v0));
        if (name == "content-length") {
          clen = atoll(val.c_str());
        } else if (name == "transfer-encoding") {
          chunked = val.find("chunked") != std::string::npos;
        } else if (name == "connection") {
          if (val.find("close") != std::string::npos) keep_alive = false;
          else if (val.find("keep-alive") != std::string::npos) keep_alive = true;
        }
      }
      if (chunked) {
        http_reply(c, 501, "{\"detail\":\"chunked bodies are not supported: send Content-Length\"}", false);
        return;
      }
      if (clen < 0 || (size_t)clen > kHttpMaxBody) {
        http_reply(c, 413, "{\"detail\":\"Content Too Large\"}", false);
        return;
      }
      if (avail < hlen + (size_t)clen) return;  // the rest of the body has not arrived yet
      const std::string body(base + hlen, (size_t)clen);
      c.in_off += hlen + (size_t)clen;
      const size_t q = path.find('?');
      if (q != std::string::npos) path.resize(q);
      http_route(c, method, path, body, keep_alive);
    }
  }

  void http_route(Conn& c, const std::string& method, const std::string& path, const std::string& body,
                  bool keep_alive) {
    const bool one = path == "/sms/raw", batch = path == "/sms/raw/batch";
    if (one || batch) {
      if (method != "POST") {
        http_reply(c, 405, "{\"detail\":\"Method Not Allowed\"}", keep_alive);
        return;
      }
      ingest::Result r = ingest::handle(body, batch);
      if (r.status == 202) {
        try {
          for (auto& raw : r.raws) eng_.store("sms.raw", std::move(raw), mp::Value::nil());
        } catch (std::exception&) {
          r.status = 500;
          r.body = "{\"detail\":\"Internal error\"}";
        }
      }
      ++http_counts_[{path, r.status}];
      http_reply(c, r.status, r.body, keep_alive);
    } else if (path == "/health" && method == "GET") {
      http_reply(c, 200, "{\"status\":\"ok\"}", keep_alive);  // this process IS the bus
    } else if (path == "/metrics" && method == "GET") {
      std::string o = "# HELP api_gateway_requests_total HTTP requests\n# TYPE api_gateway_requests_total counter\n";
      for (auto& kv : http_counts_)
        o += "api_gateway_requests_total{endpoint=\"" + kv.first.first + "\",status=\"" +
             std::to_string(kv.first.second) + "\"} " + std::to_string(kv.second) + "\n";
      http_reply(c, 200, o, keep_alive, "text/plain; version=0.0.4");
    } else {
      http_reply(c, 404, "{\"detail\":\"Not Found\"}", keep_alive);
    }
  }

  std::map<std::pair<std::string, int>, long long> http_counts_;  // (endpoint, status) -> requests

  // =================================================================== NATS

  // NATS client protocol + the JetStream API subset of bus/nats_server.py (the
  // Python front-end; tests/test_bus_nats.py runs the same client tests against
  // both): core INFO/CONNECT/PING/PONG/PUB/HPUB/SUB (queue groups)/UNSUB with
  // subject routing; a publish to a stream subject is stored (PubAck JSON to its
  // reply); $JS.API STREAM.NAMES/LIST/INFO/CREATE/UPDATE/DELETE, CONSUMER.CREATE /
  // DURABLE.CREATE / INFO / DELETE / MSG.NEXT (pull; 404 / 408 status frames) and
  // push consumers (deliver_subject); acks on $JS.ACK.* (+ACK, -NAK {delay}, +TERM,
  // +WPI, +NXT).  All on the same event loop and engine as the msgpack protocol.
  static constexpr size_t kNatsMaxPayload = 8u << 20;

  static bool starts_with(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }

  static std::vector<std::string> split_on(const std::string& s, char sep) {
    std::vector<std::string> out;
    size_t b = 0;
    for (;;) {
      size_t e = s.find(sep, b);
      out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
      if (e == std::string::npos) return out;
      b = e + 1;
    }
  }

  static std::vector<std::string> split_ws(const std::string& s) {
    std::vector<std::string> out;
    size_t k = 0;
    while (k < s.size()) {
      while (k < s.size() && (s[k] == ' ' || s[k] == '\t')) ++k;
      size_t b = k;
      while (k < s.size() && s[k] != ' ' && s[k] != '\t') ++k;
      if (k > b) out.push_back(s.substr(b, k - b));
    }
    return out;
  }

  void nats_info(Conn& c) {
    mp::Value info = mp::Value::map();
    info.put("server_id", mp::Value::str(server_id_));
    info.put("server_name", mp::Value::str("smsgate-busd"));
    info.put("version", mp::Value::str("2.10.0"));
    info.put("proto", mp::Value::integer(1));
    info.put("go", mp::Value::str("n/a"));
    info.put("host", mp::Value::str("0.0.0.0"));
    info.put("port", mp::Value::integer(nats_port_));
    info.put("headers", mp::Value::boolean(true));
    info.put("max_payload", mp::Value::integer((int64_t)kNatsMaxPayload));
    info.put("jetstream", mp::Value::boolean(true));
    c.out += "INFO " + json::dumps(info) + "\r\n";
  }

  void nats_parse(Conn& c) {
    while (!c.dead) {
      const char* base = c.in.data() + c.in_off;
      size_t avail = c.in.size() - c.in_off;
      const char* nl = (const char*)memmem(base, avail, "\r\n", 2);
      if (!nl) {
        if (avail > 64 * 1024) c.dead = true;  // no control line is this long
        return;
      }
      size_t llen = (size_t)(nl - base);
      std::string line(base, llen);
      size_t sp = line.find(' ');
      std::string op = line.substr(0, sp);
      for (auto& ch : op) ch = (char)toupper((unsigned char)ch);
      std::vector<std::string> args = split_ws(sp == std::string::npos ? std::string() : line.substr(sp + 1));
      if (op == "PUB" || op == "HPUB") {
        bool h = op == "HPUB";
        size_t need = h ? 3 : 2;
        if (args.size() != need && args.size() != need + 1) {
          c.out += "-ERR 'Unknown Protocol Operation'\r\n";
          c.dead = true;
          return;
        }
        size_t total = strtoull(args.back().c_str(), nullptr, 10);
        size_t hsize = h ? strtoull(args[args.size() - 2].c_str(), nullptr, 10) : 0;
        if (total > kNatsMaxPayload || hsize > total) {
          c.out += "-ERR 'Maximum Payload Violation'\r\n";
          c.dead = true;
          return;
        }
        if (avail < llen + 2 + total + 2) return;  // payload not complete yet
        const char* body = nl + 2;
        std::string subject = args[0];
        std::string reply = args.size() == need + 1 ? args[1] : std::string();
        std::string hdr(body, hsize), payload(body + hsize, total - hsize);
        c.in_off += llen + 2 + total + 2;
        nats_pub(subject, reply, hdr, payload);
        continue;
      }
      c.in_off += llen + 2;
      if (op == "SUB" && (args.size() == 2 || args.size() == 3)) {
        c.subs[args.back()] = NSub{args[0], args.size() == 3 ? args[1] : std::string()};
      } else if (op == "UNSUB" && !args.empty()) {
        c.subs.erase(args[0]);
      } else if (op == "PING") {
        c.out += "PONG\r\n";
      } else if (op == "CONNECT" || op == "PONG" || op == "+OK" || op.empty()) {
      } else {
        c.out += "-ERR 'Unknown Protocol Operation'\r\n";
      }
    }
  }

  static void msg_frame(std::string& o, const std::string& subject, const std::string& sid, const std::string& reply,
                        const std::string& hdr, const std::string& payload) {
    o += hdr.empty() ? "MSG " : "HMSG ";
    o += subject;
    o += ' ';
    o += sid;
    if (!reply.empty()) {
      o += ' ';
      o += reply;
    }
    if (!hdr.empty()) {
      o += ' ';
      o += std::to_string(hdr.size());
    }
    o += ' ';
    o += std::to_string(hdr.size() + payload.size());
    o += "\r\n";
    o += hdr;
    o += payload;
    o += "\r\n";
  }

  // deliver to every matching plain subscription and one member of each queue group
  int nats_route(const std::string& subject, const std::string& payload, const std::string& reply = std::string(),
                 const std::string& hdr = std::string()) {
    int n = 0;
    route_q_.clear();
    for (auto& kv : conns_) {
      Conn& c = kv.second;
      if (!c.nats || c.dead) continue;
      for (auto& sv : c.subs)
        if (bus::subject_matches(sv.second.subject, subject)) {
          if (sv.second.queue.empty()) {
            msg_frame(c.out, subject, sv.first, reply, hdr, payload);
            ++n;
          } else {
            route_q_.push_back({&sv.second.queue, {&c, &sv.first}});
          }
        }
    }
    if (!route_q_.empty()) {  // one member per queue group, round robin
      std::stable_sort(route_q_.begin(), route_q_.end(),
                       [](const QMember& x, const QMember& y) { return *x.first < *y.first; });
      for (size_t b = 0; b < route_q_.size();) {
        size_t e = b;
        while (e < route_q_.size() && *route_q_[e].first == *route_q_[b].first) ++e;
        auto& pick = route_q_[b + (rr_++) % (e - b)].second;
        msg_frame(pick.first->out, subject, *pick.second, reply, hdr, payload);
        ++n;
        b = e;
      }
    }
    return n;
  }

  bool nats_has_subscriber(const std::string& subject) {
    for (auto& kv : conns_)
      if (kv.second.nats && !kv.second.dead)
        for (auto& sv : kv.second.subs)
          if (bus::subject_matches(sv.second.subject, subject)) return true;
    return false;
  }

  void nats_status(const std::string& reply, int code, const char* text) {
    nats_route(reply, std::string(), std::string(), "NATS/1.0 " + std::to_string(code) + " " + text + "\r\n\r\n");
  }

  static mp::Value parse_headers(const std::string& raw) {
    mp::Value m = mp::Value::map();
    auto lines = split_on(raw, '\n');
    for (size_t k = 1; k < lines.size(); ++k) {
      std::string ln = lines[k];
      if (!ln.empty() && ln.back() == '\r') ln.pop_back();
      size_t colon = ln.find(':');
      if (ln.empty() || colon == std::string::npos) continue;
      auto trim = [](std::string x) {
        size_t a = x.find_first_not_of(" \t"), b = x.find_last_not_of(" \t");
        return a == std::string::npos ? std::string() : x.substr(a, b - a + 1);
      };
      m.put(trim(ln.substr(0, colon)).c_str(), mp::Value::str(trim(ln.substr(colon + 1))));
    }
    return m;
  }

  static std::string encode_headers(const mp::Value& h) {
    if (h.t != mp::Value::MAP || h.m.empty()) return std::string();
    std::string o = "NATS/1.0\r\n";
    for (auto& kv : h.m) {
      if (kv.first.t != mp::Value::STR || (kv.second.t != mp::Value::STR && kv.second.t != mp::Value::BIN)) continue;
      o += kv.first.s + ": " + kv.second.s + "\r\n";
    }
    return o + "\r\n";
  }

  void nats_pub(const std::string& subject, const std::string& reply, const std::string& hdr,
                const std::string& payload) {
    if (starts_with(subject, "$JS.API.")) {
      nats_api(subject.substr(8), payload, reply);
      return;
    }
    if (starts_with(subject, "$JS.ACK.")) {
      nats_ack(subject, payload);
      if (!reply.empty()) nats_route(reply, std::string());
      return;
    }
    bool captured = true;
    try {
      eng_.route(subject);
    } catch (bus::BusError&) {
      captured = false;
    }
    if (captured) {
      std::string data = payload;
      auto r = eng_.store(subject, std::move(data), hdr.empty() ? mp::Value::nil() : parse_headers(hdr));
      if (!reply.empty()) {
        std::string ack = "{\"stream\":";
        json::dump_str(ack, *r.first);
        ack += ",\"seq\":" + std::to_string(r.second) + "}";
        nats_route(reply, ack);
      }
    }
    int n = nats_route(subject, payload, captured ? std::string() : reply, hdr);
    if (!captured && n == 0 && !reply.empty()) nats_status(reply, 503, "No Responders");
  }

  void nats_ack(const std::string& subject, const std::string& body) {
    auto t = split_on(subject, '.');
    std::string st, cn, sseq;
    if (t.size() == 9) {
      st = t[2], cn = t[3], sseq = t[5];
    } else if (t.size() >= 11) {
      st = t[4], cn = t[5], sseq = t[7];
    } else {
      return;
    }
    int64_t seq = strtoll(sseq.c_str(), nullptr, 10);
    try {
      if (body.empty() || starts_with(body, "+ACK") || starts_with(body, "+NXT")) {
        eng_.ack(st, cn, seq);
      } else if (starts_with(body, "-NAK")) {
        double delay = 0.0;
        size_t b = body.find('{');
        if (b != std::string::npos) {
          try {
            mp::Value d = json::parse(body.substr(b));
            if (auto v = d.get("delay")) delay = v->as_double() / 1e9;
          } catch (std::exception&) {
          }
        }
        eng_.nak(st, cn, seq, delay, wall_now());
      } else if (starts_with(body, "+TERM")) {
        eng_.ack(st, cn, seq, "term");
      } else if (starts_with(body, "+WPI")) {
        eng_.touch(st, cn, seq, wall_now());
      }
    } catch (bus::BusError&) {  // ack for a deleted consumer / unknown seq: ignored, as nats-server does
    }
  }

  std::string ack_subject(const std::string& stream, const std::string& durable, const bus::Delivery& d) {
    int64_t cseq = ++cseq_[{stream, durable}];
    return "$JS.ACK." + stream + "." + durable + "." + std::to_string(d.num_delivered) + "." +
           std::to_string(d.msg->seq) + "." + std::to_string(cseq) + "." +
           std::to_string((int64_t)(d.msg->ts * 1e9)) + ".0";
  }

  int nats_deliver(const std::string& to, const std::string& stream, const std::string& durable,
                   const bus::Delivery& d) {
    return nats_route(to, d.msg->data, ack_subject(stream, durable, d), encode_headers(d.msg->headers));
  }

  static mp::Value api_error(int code, int err, const std::string& desc) {
    mp::Value e = mp::Value::map();
    e.put("code", mp::Value::integer(code));
    e.put("err_code", mp::Value::integer(err));
    e.put("description", mp::Value::str(desc));
    mp::Value v = mp::Value::map();
    v.put("error", std::move(e));
    return v;
  }

  mp::Value stream_json(const std::string& name) {
    bus::Stream& st = eng_.stream(name);
    mp::Value cfg = mp::Value::map();
    cfg.put("name", mp::Value::str(st.cfg.name));
    mp::Value subs = mp::Value::arr();
    for (auto& x : st.cfg.subjects) subs.push(mp::Value::str(x));
    cfg.put("subjects", std::move(subs));
    cfg.put("retention", mp::Value::str("limits"));
    cfg.put("max_consumers", mp::Value::integer(-1));
    cfg.put("max_msgs", mp::Value::integer(st.cfg.max_msgs));
    cfg.put("max_bytes", mp::Value::integer(st.cfg.max_bytes));
    cfg.put("max_age", mp::Value::integer((int64_t)(st.cfg.max_age * 1e9)));
    cfg.put("max_msg_size", mp::Value::integer(-1));
    cfg.put("storage", mp::Value::str(st.cfg.storage));
    cfg.put("discard", mp::Value::str("old"));
    cfg.put("num_replicas", mp::Value::integer(1));
    mp::Value state = mp::Value::map();
    state.put("messages", mp::Value::integer(st.count));
    state.put("bytes", mp::Value::integer(st.bytes));
    state.put("first_seq", mp::Value::integer(st.first_seq));
    state.put("last_seq", mp::Value::integer(st.last_seq));
    state.put("consumer_count", mp::Value::integer((int64_t)st.consumers.size()));
    mp::Value v = mp::Value::map();
    v.put("type", mp::Value::str("io.nats.jetstream.api.v1.stream_info_response"));
    v.put("config", std::move(cfg));
    v.put("created", mp::Value::str("1970-01-01T00:00:00Z"));
    v.put("state", std::move(state));
    return v;
  }

  mp::Value consumer_json(const std::string& stream, const std::string& durable) {
    mp::Value ci = eng_.consumer_info(stream, durable);
    bus::Consumer& c = eng_.consumer(stream, durable);
    auto num = [&](const char* k) { return ci.get(k)->as_int(); };
    mp::Value cfg = mp::Value::map();
    cfg.put("durable_name", mp::Value::str(durable));
    cfg.put("name", mp::Value::str(durable));
    cfg.put("ack_policy", mp::Value::str("explicit"));
    cfg.put("deliver_policy", mp::Value::str(c.cfg.deliver_policy));
    cfg.put("filter_subject", mp::Value::str(c.cfg.filter_subject));
    cfg.put("ack_wait", mp::Value::integer((int64_t)(c.cfg.ack_wait * 1e9)));
    cfg.put("max_deliver", mp::Value::integer(c.cfg.max_deliver));
    cfg.put("max_ack_pending", mp::Value::integer(c.cfg.max_ack_pending));
    cfg.put("replay_policy", mp::Value::str("instant"));
    auto it = push_.find({stream, durable});
    if (it != push_.end()) cfg.put("deliver_subject", mp::Value::str(it->second));
    auto seqs = [](int64_t cs, int64_t ss) {
      mp::Value v = mp::Value::map();
      v.put("consumer_seq", mp::Value::integer(cs));
      v.put("stream_seq", mp::Value::integer(ss));
      return v;
    };
    mp::Value v = mp::Value::map();
    v.put("type", mp::Value::str("io.nats.jetstream.api.v1.consumer_info_response"));
    v.put("stream_name", mp::Value::str(stream));
    v.put("name", mp::Value::str(durable));
    v.put("created", mp::Value::str("1970-01-01T00:00:00Z"));
    v.put("config", std::move(cfg));
    auto cs = cseq_.find({stream, durable});
    v.put("delivered", seqs(cs == cseq_.end() ? 0 : cs->second, num("delivered_seq")));
    v.put("ack_floor", seqs(0, num("ack_floor")));
    v.put("num_ack_pending", mp::Value::integer(num("num_ack_pending")));
    v.put("num_redelivered", mp::Value::integer(num("num_redelivered")));
    v.put("num_waiting", mp::Value::integer(0));
    v.put("num_pending", mp::Value::integer(num("num_pending")));
    return v;
  }

  void nats_api(const std::string& what, const std::string& body, const std::string& reply) {
    mp::Value res;
    bool answer = true;
    try {
      answer = nats_api_call(what, body, reply, res);
    } catch (bus::BusError& e) {
      std::string msg = e.what();
      bool nf = msg.find("not found") != std::string::npos;
      res = api_error(nf ? 404 : 400, nf ? (starts_with(msg, "consumer") ? 10014 : 10059) : 10058, msg);
    } catch (std::exception& e) {
      res = api_error(400, 10025, std::string("bad request: ") + e.what());
    }
    if (answer && !reply.empty()) nats_route(reply, json::dumps(res));
  }

  bus::StreamConfig stream_cfg_json(const mp::Value& d, const std::string& name) {
    bus::StreamConfig cfg;
    const mp::Value* v;
    cfg.name = (v = d.get("name")) ? v->as_str() : name;
    if ((v = d.get("subjects")) && v->t == mp::Value::ARR && !v->a.empty()) {
      for (auto& x : v->a) cfg.subjects.push_back(x.as_str());
    } else {
      cfg.subjects.push_back(cfg.name);
    }
    cfg.max_age = (v = d.get("max_age")) && !v->is_nil() ? v->as_double() / 1e9 : 0.0;
    cfg.max_msgs = (v = d.get("max_msgs")) && !v->is_nil() ? v->as_int() : -1;
    cfg.max_bytes = (v = d.get("max_bytes")) && !v->is_nil() ? v->as_int() : -1;
    cfg.storage = (v = d.get("storage")) && v->t == mp::Value::STR ? v->s : std::string("file");
    return cfg;
  }

  // false: nothing to answer now (pull requests answer with deliveries / status frames)
  bool nats_api_call(const std::string& what, const std::string& body, const std::string& reply, mp::Value& res) {
    auto t = split_on(what, '.');
    mp::Value req = mp::Value::map();
    size_t b0 = body.find_first_not_of(" \t\r\n");
    if (b0 != std::string::npos && body[b0] == '{') req = json::parse(body);
    auto tok = [&](size_t k) -> const std::string& {
      if (k >= t.size()) throw std::runtime_error("missing name in " + what);
      return t[k];
    };
    if (t[0] == "INFO") {
      res = mp::Value::map();
      res.put("type", mp::Value::str("io.nats.jetstream.api.v1.account_info_response"));
      res.put("streams", mp::Value::integer((int64_t)eng_.streams.size()));
      return true;
    }
    if (t[0] == "STREAM") {
      const std::string& op = tok(1);
      if (op == "NAMES" || op == "LIST") {
        const mp::Value* sv = req.get("subject");
        std::string subj = sv && sv->t == mp::Value::STR ? sv->s : std::string();
        mp::Value names = mp::Value::arr();
        for (auto& nm : eng_.order) {
          bool hit = subj.empty();
          for (auto& p : eng_.stream(nm).cfg.subjects)
            hit = hit || bus::subject_matches(p, subj) || bus::subject_matches(subj, p);
          if (hit) names.push(op == "LIST" ? stream_json(nm) : mp::Value::str(nm));
        }
        res = mp::Value::map();
        res.put("total", mp::Value::integer((int64_t)names.a.size()));
        res.put("offset", mp::Value::integer(0));
        res.put("limit", mp::Value::integer(1024));
        res.put("streams", std::move(names));
        return true;
      }
      const std::string& name = tok(2);
      if (op == "INFO") {
        res = stream_json(name);
      } else if (op == "CREATE" || op == "UPDATE") {
        if (op == "UPDATE") eng_.stream(name);  // must exist
        eng_.add_or_update_stream(stream_cfg_json(req, name));
        res = stream_json(name);
      } else if (op == "DELETE") {
        for (auto it = push_.begin(); it != push_.end();) it = it->first.first == name ? push_.erase(it) : std::next(it);
        eng_.delete_stream(name);
        res = mp::Value::map();
        res.put("success", mp::Value::boolean(true));
      } else {
        throw std::runtime_error("unsupported API " + what);
      }
      return true;
    }
    if (t[0] == "CONSUMER") {
      const std::string& op = tok(1);
      if (op == "CREATE" || op == "DURABLE") {
        std::string stream, name;
        if (op == "DURABLE") {  // DURABLE.CREATE.<stream>.<durable>
          stream = tok(3);
          name = tok(4);
        } else {  // CREATE.<stream>[.<consumer>[.<filter>]]
          stream = tok(2);
          if (t.size() > 3) name = t[3];
        }
        const mp::Value* c = req.get("config");
        mp::Value empty = mp::Value::map();
        if (!c || c->t != mp::Value::MAP) c = &empty;
        const mp::Value* v;
        std::string durable = (v = c->get("durable_name")) && v->t == mp::Value::STR ? v->s
                              : (v = c->get("name")) && v->t == mp::Value::STR ? v->s : name;
        if (durable.empty()) throw std::runtime_error("ephemeral consumers are not supported");
        bus::ConsumerConfig cc;
        cc.durable = durable;
        if ((v = c->get("filter_subject")) && v->t == mp::Value::STR && !v->s.empty()) cc.filter_subject = v->s;
        if ((v = c->get("ack_wait")) && !v->is_nil()) cc.ack_wait = v->as_double() / 1e9;
        if ((v = c->get("max_deliver")) && !v->is_nil()) cc.max_deliver = v->as_int();
        if ((v = c->get("deliver_policy")) && v->t == mp::Value::STR &&
            (v->s == "all" || v->s == "new" || v->s == "last"))
          cc.deliver_policy = v->s;
        if ((v = c->get("max_ack_pending")) && !v->is_nil() && v->as_int() > 0) cc.max_ack_pending = v->as_int();
        eng_.add_consumer(stream, cc);
        if ((v = c->get("deliver_subject")) && v->t == mp::Value::STR && !v->s.empty())
          push_[{stream, durable}] = v->s;
        res = consumer_json(stream, durable);
        return true;
      }
      if (op == "INFO") {
        res = consumer_json(tok(2), tok(3));
        return true;
      }
      if (op == "DELETE") {
        push_.erase({tok(2), tok(3)});
        eng_.delete_consumer(tok(2), tok(3));
        res = mp::Value::map();
        res.put("success", mp::Value::boolean(true));
        return true;
      }
      if (op == "MSG" && tok(2) == "NEXT") {
        nats_pull(tok(3), tok(4), body, req, reply);
        return false;
      }
    }
    throw std::runtime_error("unsupported API " + what);
  }

  void nats_pull(const std::string& stream, const std::string& durable, const std::string& body,
                 const mp::Value& req, const std::string& reply) {
    if (reply.empty()) return;
    eng_.consumer(stream, durable);  // BusError -> error JSON to the requester
    NWaiter w;
    w.reply = reply;
    w.stream = stream;
    w.durable = durable;
    int64_t batch = 1;
    double expires = 0.0;
    bool no_wait = false;
    const mp::Value* v;
    if (req.t == mp::Value::MAP && !req.m.empty()) {
      if ((v = req.get("batch")) && !v->is_nil()) batch = v->as_int();
      if ((v = req.get("expires")) && !v->is_nil()) expires = v->as_double() / 1e9;
      if ((v = req.get("no_wait"))) no_wait = v->t == mp::Value::BOOL ? v->b : v->as_int() != 0;
    } else {
      size_t b0 = body.find_first_not_of(" \t\r\n");
      if (b0 != std::string::npos) batch = strtoll(body.c_str() + b0, nullptr, 10);
    }
    w.batch = std::max<int64_t>(1, batch);
    w.no_wait = no_wait || expires <= 0;
    double now = wall_now();
    w.deadline = now + (w.no_wait ? 0.0 : expires);
    if (!serve_pull(w, now)) nwaiters_.push_back(std::move(w));
  }

  // true = the pull request is finished (filled, or answered with a status frame)
  bool serve_pull(NWaiter& w, double now) {
    auto got = eng_.next_batch(w.stream, w.durable, w.batch - w.sent, now);
    for (auto& d : got) nats_deliver(w.reply, w.stream, w.durable, d);
    w.sent += (int64_t)got.size();
    if (w.sent >= w.batch) return true;
    if (w.no_wait) {  // what was there has been sent: end the request
      nats_status(w.reply, 404, "No Messages");
      return true;
    }
    if (now >= w.deadline) {
      nats_status(w.reply, 408, "Request Timeout");
      return true;
    }
    return false;
  }

  void serve_nats(double now) {
    for (auto it = nwaiters_.begin(); it != nwaiters_.end();) {
      bool done;
      try {
        done = serve_pull(*it, now);
      } catch (std::exception&) {
        nats_status(it->reply, 409, "Consumer Deleted");
        done = true;
      }
      it = done ? nwaiters_.erase(it) : std::next(it);
    }
    for (auto it = push_.begin(); it != push_.end();) {
      const std::string& st = it->first.first;
      const std::string& du = it->first.second;
      try {
        if (nats_has_subscriber(it->second)) {
          auto got = eng_.next_batch(st, du, 256, now);
          for (auto& d : got)
            if (nats_deliver(it->second, st, du, d) == 0) eng_.nak(st, du, d.msg->seq, 0.0, now);
        }
        ++it;
      } catch (std::exception&) {
        it = push_.erase(it);  // consumer / stream gone
      }
    }
  }

  bus::Engine& eng_;
  Journal* jr_;
  double max_age_;
  int ep_;
  std::vector<int> listeners_;
  std::unordered_map<uint64_t, Conn> conns_;
  std::list<Waiter> waiters_;
  std::list<NWaiter> nwaiters_;
  using QMember = std::pair<const std::string*, std::pair<Conn*, const std::string*>>;  // queue, (conn, sid)
  std::vector<QMember> route_q_;
  std::map<std::pair<std::string, std::string>, std::string> push_;  // push consumer -> deliver subject
  std::map<std::pair<std::string, std::string>, int64_t> cseq_;      // consumer sequence (ack subjects)
  uint64_t rr_ = 0;                                                   // queue-group round robin
  std::string server_id_ = "NSMSGATEBUSD" + std::to_string(getpid());

 public:
  int nats_port_ = 4222;

 private:
  uint64_t next_id_ = 0;
  double last_expire_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> listens, nats_listens, http_listens;
  std::string data_dir, fsync_mode = "interval";
  double max_age = 3 * 24 * 3600.0, fsync_interval = 0.05;
  int64_t compact_bytes = 256ll << 20;
  for (int k = 1; k < argc; ++k) {
    std::string a = argv[k];
    auto val = [&]() -> std::string {
      if (k + 1 >= argc) die("missing value for " + a);
      return argv[++k];
    };
    if (a == "--listen") listens.push_back(val());
    else if (a == "--nats-listen") nats_listens.push_back(val());
    else if (a == "--http-listen") http_listens.push_back(val());
    else if (a == "--data") data_dir = val();
    else if (a == "--max-age") max_age = atof(val().c_str());
    else if (a == "--fsync") fsync_mode = val();
    else if (a == "--fsync-interval") fsync_interval = atof(val().c_str());
    else if (a == "--compact-bytes") compact_bytes = atoll(val().c_str());
    else if (a == "-h" || a == "--help") {
      printf("usage: smsgate-busd --listen URL [--listen URL] [--nats-listen tcp://HOST:PORT] "
             "[--http-listen tcp://HOST:PORT] [--data DIR] [--max-age S] "
             "[--fsync interval|always|never] [--fsync-interval S] [--compact-bytes N]\n");
      return 0;
    } else die("unknown argument " + a);
  }
  if (listens.empty() && nats_listens.empty() && http_listens.empty()) listens.push_back("tcp://127.0.0.1:4222");
  if (fsync_mode != "interval" && fsync_mode != "always" && fsync_mode != "never") die("bad --fsync " + fsync_mode);

  struct sigaction sa{};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);

  bus::Engine eng(wall_now);
  std::unique_ptr<Journal> jr;
  if (!data_dir.empty()) {
    jr.reset(new Journal(data_dir, fsync_mode, fsync_interval, compact_bytes));
    recover(eng, *jr);
    Journal* j = jr.get();
    eng.journal = [j](const char* kind, mp::Value&& args) { j->append(kind, std::move(args)); };
    eng.fast = j;
  }
  Server srv(eng, jr.get(), max_age);
  if (eng.streams.empty()) eng.add_or_update_stream(srv.default_config());
  if (jr) jr->flush();
  int tcp_port = -1;
  for (auto& l : listens) {
    int p = srv.listen_on(l);
    if (p >= 0 && tcp_port < 0) tcp_port = p;
  }
  int nats_port = -1;
  for (auto& l : nats_listens) {
    int p = srv.listen_on(l, true);
    if (p >= 0 && nats_port < 0) nats_port = srv.nats_port_ = p;
  }
  int http_port = -1;
  for (auto& l : http_listens) {
    int p = srv.listen_on(l, false, true);
    if (p >= 0 && http_port < 0) http_port = p;
  }
  std::string ready = tcp_port >= 0 ? "READY " + std::to_string(tcp_port) : std::string("READY -");
  if (nats_port >= 0) ready += " NATS " + std::to_string(nats_port);
  if (http_port >= 0) ready += " HTTP " + std::to_string(http_port);
  printf("%s\n", ready.c_str());
  fflush(stdout);
  srv.run();
  return 0;
}
