// smsgate-busload — native load generator for the bus broker (capacity tests).
//
// Python clients cannot saturate a C++ broker on a few cores, so broker
// capacity is measured with this: P producer threads each publish N messages of
// --payload bytes to --subject in publish_many frames of --batch, with up to
// --depth frames in flight per connection; C consumer threads share ONE durable
// competing group, fetch --fetch messages at a time and ack them with one
// ack_many frame.  Every thread has its own connection (the broker's view is
// P + C clients, as with P gateway and C parser processes).  Timing runs from
// the first publish to the moment the consumers have acked every message.
//
// Usage: smsgate-busload --socket /path/bus.sock [--producers 4] [--consumers 64]
//                        [--msgs 100000] [--batch 256] [--fetch 256] [--depth 4]
//                        [--payload 300] [--durable load]
// Prints one JSON line: {"published":..,"acked":..,"seconds":..,"publish_per_s":..}
//
// HTTP mode (the broker's native ingestion front-end, --http-listen):
//   smsgate-busload --http PORT [--path /sms/raw] [--conns 64] [--seconds 5] [--depth 1] [--batch 1]
// C threads, one keep-alive connection each, keep --depth requests in flight
// (pipelined) and count 202 answers for --seconds; --batch > 1 posts
// /sms/raw/batch arrays.  Prints {"mode":"http","requests_per_s":..,"msgs_per_s":..}.
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mpack.hpp"

namespace {

struct Opts {
  std::string socket, path = "/sms/raw";
  int http_port = 0, conns = 64;
  double seconds = 5.0;
  int producers = 4, consumers = 64, batch = 256, fetch = 256, depth = 4, payload = 300;
  long msgs = 100000;
  std::string durable = "load", subject = "sms.raw", stream = "SMS";
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int dial(const std::string& path) {
  int fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  sockaddr_un a{};
  a.sun_family = AF_UNIX;
  strncpy(a.sun_path, path.c_str(), sizeof(a.sun_path) - 1);
  if (::connect(fd, (sockaddr*)&a, sizeof(a)) < 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

bool send_all(int fd, const std::string& b) {
  size_t off = 0;
  while (off < b.size()) {
    ssize_t w = ::write(fd, b.data() + off, b.size() - off);
    if (w <= 0) return false;
    off += (size_t)w;
  }
  return true;
}

bool read_exact(int fd, char* p, size_t n) {
  while (n) {
    ssize_t r = ::read(fd, p, n);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

// one reply frame -> decoded [rid, ok, result]
bool read_reply(int fd, mp::Value& out) {
  uint32_t n;
  if (!read_exact(fd, (char*)&n, 4)) return false;  // little-endian length (x86)
  std::string body(n, '\0');
  if (!read_exact(fd, &body[0], n)) return false;
  out = mp::decode(body.data(), body.size());
  return out.t == mp::Value::ARR && out.a.size() >= 3 && out.a[1].t == mp::Value::BOOL && out.a[1].b;
}

std::string frame(const std::string& body) {
  std::string f;
  uint32_t n = (uint32_t)body.size();
  f.append((const char*)&n, 4);
  f += body;
  return f;
}

std::string req_hdr(const char* op, int64_t rid, size_t nargs) {
  std::string o;
  mp::enc_arr_hdr(o, 2 + nargs);
  mp::enc_str(o, op, strlen(op));
  mp::enc_int(o, rid);
  return o;
}

bool call(int fd, std::string body, mp::Value& rep) { return send_all(fd, frame(body)) && read_reply(fd, rep); }

std::atomic<long> g_acked{0}, g_published{0};
std::atomic<bool> g_go{false}, g_fail{false};

void producer(const Opts& o, int idx) {
  int fd = dial(o.socket);
  if (fd < 0) { g_fail = true; return; }
  std::string pay(o.payload, 'x');
  while (!g_go.load()) std::this_thread::yield();
  long sent = 0, inflight = 0;
  int64_t rid = 1;
  mp::Value rep;
  while (sent < o.msgs || inflight) {
    while (sent < o.msgs && inflight < o.depth) {
      const long k = std::min<long>(o.batch, o.msgs - sent);
      std::string b = req_hdr("publish_many", rid++, 1);
      mp::enc_arr_hdr(b, (size_t)k);
      for (long i = 0; i < k; ++i) {
        mp::enc_arr_hdr(b, 2);
        mp::enc_str(b, o.subject);
        snprintf(&pay[0], 24, "%08d-%012ld", idx, sent + i);
        mp::enc_bin(b, pay.data(), pay.size());
      }
      if (!send_all(fd, frame(b))) { g_fail = true; return; }
      sent += k;
      ++inflight;
    }
    if (!read_reply(fd, rep)) { g_fail = true; return; }
    g_published += (long)rep.a[2].a.size();
    --inflight;
  }
  ::close(fd);
}

void consumer(const Opts& o, long total) {
  int fd = dial(o.socket);
  if (fd < 0) { g_fail = true; return; }
  mp::Value rep;
  {
    std::string b = req_hdr("subscribe", 1, 3);
    mp::enc_str(b, o.subject);
    mp::enc_str(b, o.durable);
    mp::enc_map_hdr(b, 0);
    if (!call(fd, b, rep)) { g_fail = true; return; }
  }
  int64_t rid = 2;
  while (g_acked.load() < total && !g_fail.load()) {
    std::string b = req_hdr("fetch", rid++, 4);
    mp::enc_str(b, o.stream);
    mp::enc_str(b, o.durable);
    mp::enc_int(b, o.fetch);
    mp::enc_double(b, 0.05);
    if (!call(fd, b, rep)) { g_fail = true; return; }
    const auto& rows = rep.a[2].a;
    if (rows.empty()) continue;
    std::string ack = req_hdr("ack_many", 0, 3);  // fire-and-forget
    mp::enc_str(ack, o.stream);
    mp::enc_str(ack, o.durable);
    mp::enc_arr_hdr(ack, rows.size());
    for (const auto& r : rows) mp::enc_int(ack, r.a[2].as_int());
    if (!send_all(fd, frame(ack))) { g_fail = true; return; }
    g_acked += (long)rows.size();
  }
  ::close(fd);
}

// ---------------------------------------------------------------- HTTP mode
std::atomic<long> g_http_ok{0}, g_http_msgs{0}, g_http_other{0};

std::string http_request(const Opts& o, long k) {
  std::string body;
  auto one = [&](long i) {
    return std::string("{\"device_id\":\"load\",\"message\":\"APPROVED PURCHASE DB SALE: SHOP ") +
           std::to_string(i) + ", YEREVAN,06.05.25 14:23,card ***0018. Amount:" + std::to_string(i % 997 + 1) +
           ".00 USD, Balance:1842.74 USD\",\"sender\":\"BANK\",\"timestamp\":1746541380,\"source\":\"device\"}";
  };
  if (o.batch > 1) {
    body = "[";
    for (int b = 0; b < o.batch; ++b) body += (b ? "," : "") + one(k * o.batch + b);
    body += "]";
  } else {
    body = one(k);
  }
  return "POST " + o.path + " HTTP/1.1\r\nHost: load\r\nContent-Type: application/json\r\nContent-Length: " +
         std::to_string(body.size()) + "\r\n\r\n" + body;
}

void http_worker(const Opts& o, int idx, double t_end) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)o.http_port);
  a.sin_addr.s_addr = htonl(0x7f000001);
  if (fd < 0 || ::connect(fd, (sockaddr*)&a, sizeof a) < 0) { g_fail = true; return; }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  std::vector<std::string> reqs;
  for (int k = 0; k < 64; ++k) reqs.push_back(http_request(o, (long)idx * 1000000 + k));
  std::string in;
  long sent = 0, got = 0;
  char buf[1 << 16];
  while (!g_go.load()) std::this_thread::yield();
  bool stop = false;
  while (!stop || got < sent) {
    while (!stop && sent - got < o.depth) {
      if (!send_all(fd, reqs[sent % reqs.size()])) { g_fail = true; return; }
      ++sent;
      if (now_s() >= t_end) stop = true;
    }
    ssize_t r = ::read(fd, buf, sizeof buf);
    if (r <= 0) { g_fail = true; return; }
    in.append(buf, (size_t)r);
    for (;;) {  // complete responses in `in`
      size_t he = in.find("\r\n\r\n");
      if (he == std::string::npos) break;
      size_t cl = in.find("content-length: ");
      if (cl == std::string::npos || cl > he) { g_fail = true; return; }
      long clen = atol(in.c_str() + cl + 16);
      if (in.size() < he + 4 + (size_t)clen) break;
      int status = atoi(in.c_str() + 9);
      if (status == 202) { ++g_http_ok; g_http_msgs += o.batch > 1 ? o.batch : 1; }
      else ++g_http_other;
      in.erase(0, he + 4 + (size_t)clen);
      ++got;
    }
    if (now_s() >= t_end) stop = true;
  }
  ::close(fd);
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  bool batch_given = false;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--socket") o.socket = v;
    else if (k == "--producers") o.producers = atoi(v.c_str());
    else if (k == "--consumers") o.consumers = atoi(v.c_str());
    else if (k == "--msgs") o.msgs = atol(v.c_str());
    else if (k == "--batch") o.batch = atoi(v.c_str()), batch_given = true;
    else if (k == "--fetch") o.fetch = atoi(v.c_str());
    else if (k == "--depth") o.depth = atoi(v.c_str());
    else if (k == "--payload") o.payload = std::max(24, atoi(v.c_str()));
    else if (k == "--durable") o.durable = v;
    else if (k == "--http") o.http_port = atoi(v.c_str());
    else if (k == "--path") o.path = v;
    else if (k == "--conns") o.conns = atoi(v.c_str());
    else if (k == "--seconds") o.seconds = atof(v.c_str());
    else { fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
  }
  if (o.http_port > 0) {
    if (!batch_given) o.batch = 1;  // one SMS per request unless --batch is given
    if (o.batch > 1 && o.path == "/sms/raw") o.path = "/sms/raw/batch";
    const double t0 = now_s();
    std::vector<std::thread> ts;
    for (int c = 0; c < o.conns; ++c) ts.emplace_back(http_worker, std::cref(o), c, t0 + o.seconds);
    g_go = true;
    for (auto& t : ts) t.join();
    const double dt = now_s() - t0;
    printf("{\"mode\": \"http\", \"path\": \"%s\", \"conns\": %d, \"depth\": %d, \"batch\": %d, \"seconds\": %.3f, "
           "\"requests_202\": %ld, \"requests_other\": %ld, \"requests_per_s\": %.0f, \"msgs_per_s\": %.0f, "
           "\"ok\": %s}\n",
           o.path.c_str(), o.conns, o.depth, o.batch, dt, g_http_ok.load(), g_http_other.load(), g_http_ok.load() / dt,
           g_http_msgs.load() / dt, g_fail.load() ? "false" : "true");
    return g_fail.load() ? 1 : 0;
  }
  if (o.socket.empty()) { fprintf(stderr, "--socket required\n"); return 2; }
  {  // the stream must exist before consumers subscribe
    int fd = dial(o.socket);
    mp::Value rep;
    std::string b = req_hdr("ensure_stream", 1, 1);
    mp::enc_nil(b);
    if (fd < 0 || !call(fd, b, rep)) { fprintf(stderr, "cannot reach the broker\n"); return 1; }
    ::close(fd);
  }
  const long total = o.msgs * o.producers;
  std::vector<std::thread> ts;
  for (int c = 0; c < o.consumers; ++c) ts.emplace_back(consumer, std::cref(o), total);
  std::this_thread::sleep_for(std::chrono::milliseconds(300));  // subscriptions in place
  for (int p = 0; p < o.producers; ++p) ts.emplace_back(producer, std::cref(o), p);
  const double t0 = now_s();
  g_go = true;
  for (auto& t : ts) t.join();
  const double dt = now_s() - t0;
  printf("{\"published\": %ld, \"acked\": %ld, \"seconds\": %.4f, \"publish_per_s\": %.0f, \"producers\": %d, "
         "\"consumers\": %d, \"batch\": %d, \"fetch\": %d, \"payload\": %d, \"ok\": %s}\n",
         g_published.load(), g_acked.load(), dt, g_acked.load() / dt, o.producers, o.consumers, o.batch, o.fetch,
         o.payload, g_fail.load() ? "false" : "true");
  return g_fail.load() ? 1 : 0;
}
