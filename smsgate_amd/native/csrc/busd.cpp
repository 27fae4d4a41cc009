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
// Prints ``READY <tcp-port|->`` on stdout once listening.
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
#include <list>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine.hpp"

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
class Journal {
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
struct Conn {
  int fd;
  uint64_t id;
  std::string in;
  size_t in_off = 0;
  std::string out;
  size_t out_off = 0;
  bool writing = false;
  bool dead = false;
};

struct Waiter {
  uint64_t conn;
  int64_t rid;
  std::string stream, durable;
  int64_t batch;
  double deadline;  // wall clock; INFINITY = wait forever
};

const char* kAllSubjects[] = {"sms.raw", "sms.parsed", "sms.failed", "sms.processing", "sms.categorized"};

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

  int listen_on(const std::string& url) {
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
    ev.data.u64 = (uint64_t)fd | (1ull << 63);
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
          accept_all((int)(tag & 0xffffffff));
          continue;
        }
        auto it = conns_.find(tag);
        if (it == conns_.end()) continue;
        Conn& c = it->second;
        if (evs[k].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) read_conn(c);
        if (evs[k].events & EPOLLOUT) c.writing = false;  // retry the write below
      }
      double now = wall_now();
      if (now - last_expire_ >= 1.0) {
        eng_.expire(now);
        last_expire_ = now;
      }
      serve_waiters(now);
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
    if (jr_) t = std::min(t, jr_->sync_due_in());
    return (int)std::ceil(t * 1000.0);
  }

  void accept_all(int lfd) {
    for (;;) {
      int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);  // harmless failure on AF_UNIX
      uint64_t id = ++next_id_;
      Conn& c = conns_[id];
      c.fd = fd;
      c.id = id;
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
    while (c.in.size() - c.in_off >= 4) {
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
      if (c.out_off == c.out.size() && !c.out.empty()) {
        c.out.clear();
        c.out_off = 0;
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLRDHUP;
        ev.data.u64 = c.id;
        epoll_ctl(ep_, EPOLL_CTL_MOD, c.fd, &ev);
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

  bus::Engine& eng_;
  Journal* jr_;
  double max_age_;
  int ep_;
  std::vector<int> listeners_;
  std::unordered_map<uint64_t, Conn> conns_;
  std::list<Waiter> waiters_;
  uint64_t next_id_ = 0;
  double last_expire_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> listens;
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
    else if (a == "--data") data_dir = val();
    else if (a == "--max-age") max_age = atof(val().c_str());
    else if (a == "--fsync") fsync_mode = val();
    else if (a == "--fsync-interval") fsync_interval = atof(val().c_str());
    else if (a == "--compact-bytes") compact_bytes = atoll(val().c_str());
    else if (a == "-h" || a == "--help") {
      printf("usage: smsgate-busd --listen URL [--listen URL] [--data DIR] [--max-age S] "
             "[--fsync interval|always|never] [--fsync-interval S] [--compact-bytes N]\n");
      return 0;
    } else die("unknown argument " + a);
  }
  if (listens.empty()) listens.push_back("tcp://127.0.0.1:4222");
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
  }
  Server srv(eng, jr.get(), max_age);
  if (eng.streams.empty()) eng.add_or_update_stream(srv.default_config());
  if (jr) jr->flush();
  int tcp_port = -1;
  for (auto& l : listens) {
    int p = srv.listen_on(l);
    if (p >= 0 && tcp_port < 0) tcp_port = p;
  }
  if (tcp_port >= 0) printf("READY %d\n", tcp_port);
  else printf("READY -\n");
  fflush(stdout);
  srv.run();
  return 0;
}
