// HTTP/1.1 server + REST router + REST client (see sda/http.hpp).
#include "sda/http.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <sstream>

#include "sda/log.hpp"

namespace sda {

namespace {

std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}
std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  if (a == std::string::npos) return "";
  return s.substr(a, b - a + 1);
}
std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == d) { out.push_back(cur); cur.clear(); }
    else cur.push_back(c);
  }
  out.push_back(cur);
  return out;
}
bool send_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}
const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Payload Too Large";
    default: return "Internal Server Error";
  }
}

// Strict unsigned parse (digits of `base` only, no sign / whitespace / overflow).
bool parse_uint(const std::string& s, int base, size_t& out) {
  if (s.empty() || s.size() > 16) return false;
  size_t v = 0;
  for (char c : s) {
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (base == 16 && c >= 'a' && c <= 'f') d = c - 'a' + 10;
    else if (base == 16 && c >= 'A' && c <= 'F') d = c - 'A' + 10;
    else return false;
    if (v > (SIZE_MAX - (size_t)d) / (size_t)base) return false;
    v = v * (size_t)base + (size_t)d;
  }
  out = v;
  return true;
}

enum class ReadStatus { Ok, Closed, Malformed, TooLarge };

// Read one HTTP message (request or response) head + body from fd. `buf` may
// hold bytes of a following message. Never throws: a peer can make it return
// Malformed / TooLarge, nothing else.
ReadStatus read_message(int fd, std::string& buf, std::string& head, std::string& body,
                        bool is_response, size_t max_body) {
  size_t hdr_end;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    if (buf.size() > (1 << 20)) return ReadStatus::Malformed;
    char tmp[65536];
    ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return ReadStatus::Closed;
    buf.append(tmp, (size_t)r);
  }
  head = buf.substr(0, hdr_end);
  buf.erase(0, hdr_end + 4);
  std::string lh = lower(head);
  size_t clen = 0;
  bool has_len = false, chunked = false;
  for (auto& line : split(lh, '\n')) {
    auto l = trim(line);
    if (l.rfind("content-length:", 0) == 0) {
      if (!parse_uint(trim(l.substr(15)), 10, clen)) return ReadStatus::Malformed;
      has_len = true;
    } else if (l.rfind("transfer-encoding:", 0) == 0 && l.find("chunked") != std::string::npos) {
      chunked = true;
    }
  }
  auto fill = [&](size_t need) -> bool {
    while (buf.size() < need) {
      char tmp[1 << 16];
      ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) return false;
      buf.append(tmp, (size_t)r);
    }
    return true;
  };
  body.clear();
  if (chunked) {
    while (true) {
      size_t eol;
      while ((eol = buf.find("\r\n")) == std::string::npos) {
        if (buf.size() > 4096) return ReadStatus::Malformed;  // a chunk-size line is short
        if (!fill(buf.size() + 1)) return ReadStatus::Closed;
      }
      std::string size_field = buf.substr(0, eol);
      auto ext = size_field.find(';');  // chunk extensions are ignored
      if (ext != std::string::npos) size_field.resize(ext);
      size_t n;
      if (!parse_uint(trim(size_field), 16, n)) return ReadStatus::Malformed;
      // the budget is checked before anything of the chunk is buffered
      if (n > max_body || body.size() > max_body - n) return ReadStatus::TooLarge;
      buf.erase(0, eol + 2);
      if (!fill(n + 2)) return ReadStatus::Closed;
      if (buf[n] != '\r' || buf[n + 1] != '\n') return ReadStatus::Malformed;
      body.append(buf, 0, n);
      buf.erase(0, n + 2);
      if (n == 0) break;
    }
  } else if (has_len) {
    if (clen > max_body) return ReadStatus::TooLarge;
    if (buf.size() >= clen) {
      body = buf.substr(0, clen);
      buf.erase(0, clen);
    } else {
      // a long body (bulk uploads and downloads reach hundreds of megabytes) is
      // received straight into its final storage: one allocation, no staging copy
      size_t have = buf.size();
      body.swap(buf);
      buf.clear();
      body.resize(clen);
      while (have < clen) {
        ssize_t r = ::recv(fd, &body[have], clen - have, 0);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return ReadStatus::Closed;
        have += (size_t)r;
      }
    }
  } else if (is_response) {
    char tmp[1 << 16];
    while (true) {
      ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) break;
      buf.append(tmp, (size_t)r);
      if (buf.size() > max_body) return ReadStatus::TooLarge;
    }
    body.swap(buf);
  }
  return ReadStatus::Ok;
}

}  // namespace

std::string HttpRequest::header(const std::string& n) const {
  auto it = headers.find(n);
  return it == headers.end() ? "" : it->second;
}

std::string url_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%') {
      size_t v;
      if (i + 3 > s.size() || !parse_uint(s.substr(i + 1, 2), 16, v))
        throw SdaError(ErrorKind::Invalid, "malformed %-escape in URL");
      out.push_back((char)v);
      i += 2;
    } else if (s[i] == '+') {
      out.push_back(' ');
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

std::string url_encode(const std::string& s) {
  std::string out;
  char buf[4];
  for (unsigned char c : s) {
    if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
      out.push_back((char)c);
    } else {
      std::snprintf(buf, sizeof(buf), "%%%02X", c);
      out += buf;
    }
  }
  return out;
}

// ---- HttpServer -----------------------------------------------------------------
struct HttpServer::Queue {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<int> fds;
};

HttpServer::HttpServer(Handler handler, int threads)
    : handler_(std::move(handler)), threads_(std::max(1, threads)), q_(new Queue) {}

HttpServer::~HttpServer() { stop(); }

int HttpServer::start(const std::string& bind) {
  auto colon = bind.rfind(':');
  std::string host = colon == std::string::npos ? bind : bind.substr(0, colon);
  int port = colon == std::string::npos ? 8888 : std::stoi(bind.substr(colon + 1));
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw SdaError("http: socket failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0") addr.sin_addr.s_addr = INADDR_ANY;
  else if (host == "localhost") addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  else if (::inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) throw SdaError("http: bad bind address " + bind);
  if (::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
    ::close(listen_fd_);
    listen_fd_ = -1;
    throw SdaError("http: cannot bind " + bind);
  }
  if (::listen(listen_fd_, 256) != 0) throw SdaError("http: listen failed");
  socklen_t len = sizeof(addr);
  ::getsockname(listen_fd_, (sockaddr*)&addr, &len);
  port_ = ntohs(addr.sin_port);
  running_ = true;
  for (int i = 0; i < threads_; ++i) workers_.emplace_back([this] { worker_loop(); });
  acceptor_ = std::thread([this] { accept_loop(); });
  return port_;
}

void HttpServer::accept_loop() {
  while (running_) {
    pollfd p{listen_fd_, POLLIN, 0};
    int r = ::poll(&p, 1, 100);
    if (r <= 0) continue;
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    {
      std::lock_guard<std::mutex> g(q_->mu);
      q_->fds.push_back(fd);
    }
    q_->cv.notify_one();
  }
}

void HttpServer::worker_loop() {
  while (true) {
    int fd;
    {
      std::unique_lock<std::mutex> g(q_->mu);
      q_->cv.wait(g, [&] { return !q_->fds.empty() || !running_; });
      if (!running_ && q_->fds.empty()) return;
      fd = q_->fds.front();
      q_->fds.pop_front();
    }
    try {
      handle_conn(fd);
    } catch (...) {
      // a worker never dies with its connection
    }
    ::close(fd);
  }
}

void HttpServer::handle_conn(int fd) {
  std::string buf;
  while (running_) {
    std::string head, body;
    pollfd p{fd, POLLIN, 0};
    if (buf.empty() && ::poll(&p, 1, 30000) <= 0) return;  // idle keep-alive timeout
    const ReadStatus rs = read_message(fd, buf, head, body, false, max_body_);
    if (rs == ReadStatus::Closed) return;
    HttpRequest req;
    HttpResponse resp;
    bool keep_alive = false;
    // Nothing a peer sends may escape as an exception: a malformed request is
    // answered with 400 (413 for an oversized body) and the connection closed.
    bool parsed = false;
    if (rs == ReadStatus::Ok) {
      try {
        auto lines = split(head, '\n');
        auto rl = split(trim(lines.at(0)), ' ');
        if (rl.size() < 2) throw SdaError(ErrorKind::Invalid, "malformed request line");
        req.method = rl[0];
        req.target = rl[1];
        auto qpos = req.target.find('?');
        req.path = qpos == std::string::npos ? req.target : req.target.substr(0, qpos);
        if (qpos != std::string::npos) {
          for (auto& kv : split(req.target.substr(qpos + 1), '&')) {
            auto eq = kv.find('=');
            if (eq == std::string::npos) req.query[url_decode(kv)] = "";
            else req.query[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
          }
        }
        keep_alive = rl.size() >= 3 && rl[2].find("1.1") != std::string::npos;
        for (size_t i = 1; i < lines.size(); ++i) {
          auto c = lines[i].find(':');
          if (c == std::string::npos) continue;
          req.headers[lower(trim(lines[i].substr(0, c)))] = trim(lines[i].substr(c + 1));
        }
        if (lower(req.header("connection")) == "close") keep_alive = false;
        if (lower(req.header("connection")) == "keep-alive") keep_alive = true;
        req.body = std::move(body);
        parsed = true;
      } catch (const std::exception& e) {
        resp.body = e.what();
      }
    }
    if (!parsed) {
      resp.status = rs == ReadStatus::TooLarge ? 413 : 400;
      resp.content_type = "text/plain; charset=utf-8";
      if (resp.body.empty())
        resp.body = rs == ReadStatus::TooLarge ? "request body too large" : "malformed HTTP request";
      keep_alive = false;  // the stream position is unknown after a bad message
    } else {
      try {
        resp = handler_(req);
      } catch (const std::exception& e) {
        resp.status = 500;
        resp.content_type = "text/plain; charset=utf-8";
        resp.body = e.what();
      } catch (...) {
        resp.status = 500;
        resp.content_type = "text/plain; charset=utf-8";
        resp.body = "internal error";
      }
    }
    std::ostringstream out;
    out << "HTTP/1.1 " << resp.status << " " << reason(resp.status) << "\r\n";
    if (!resp.content_type.empty()) out << "Content-Type: " << resp.content_type << "\r\n";
    out << "Content-Length: " << resp.body.size() << "\r\n";
    for (auto& h : resp.headers) out << h.first << ": " << h.second << "\r\n";
    out << (keep_alive ? "Connection: keep-alive\r\n" : "Connection: close\r\n") << "\r\n";
    std::string hdr = out.str();
    if (!send_all(fd, hdr.data(), hdr.size()) || !send_all(fd, resp.body.data(), resp.body.size())) return;
    if (!keep_alive) return;
  }
}

void HttpServer::serve_forever() {
  while (running_) std::this_thread::sleep_for(std::chrono::milliseconds(200));
}

void HttpServer::stop() {
  if (!running_.exchange(false)) return;
  q_->cv.notify_all();
  if (acceptor_.joinable()) acceptor_.join();
  for (auto& w : workers_)
    if (w.joinable()) w.join();
  workers_.clear();
  if (listen_fd_ >= 0) ::close(listen_fd_);
  listen_fd_ = -1;
}

// ---- REST router ----------------------------------------------------------------
// Deviation: the reference answers 500 for a missing / malformed header (its
// errors are plain strings there); here they are InvalidCredentials -> 401.
AuthToken parse_basic_auth(const std::string& header_value) {
  auto fail = [](const char* why) { return SdaError(ErrorKind::InvalidCredentials, why); };
  std::string h = trim(header_value);
  if (h.empty()) throw fail("Mandatory Authorization header");
  if (h.rfind("Basic ", 0) != 0) throw fail("Basic Authorization required");
  Bytes dec;
  try {
    dec = base64_decode(trim(h.substr(6)));
  } catch (const SdaError&) {
    throw fail("Invalid Auth header (base64)");
  }
  std::string s(dec.begin(), dec.end());
  auto c = s.find(':');
  if (c == std::string::npos) throw fail("Invalid Auth header");
  AuthToken t;
  try {
    t.id = AgentId::parse(s.substr(0, c));
  } catch (const SdaError&) {
    throw fail("Invalid Auth header (agent id)");
  }
  t.body = s.substr(c + 1);
  return t;
}

namespace {

HttpResponse json_resp(const json::Value& v) {
  HttpResponse r;
  r.status = 200;
  r.content_type = "application/json";
  r.body = v.dump();
  return r;
}
HttpResponse not_found_resource() {
  HttpResponse r;
  r.status = 404;
  r.headers.emplace_back("Resource-not-found", "true");
  return r;
}
HttpResponse empty(int code) {
  HttpResponse r;
  r.status = code;
  return r;
}
template <class T>
HttpResponse opt_json(const std::optional<T>& v) {
  if (!v) return not_found_resource();
  return json_resp(wire::to_json(*v));
}
// A response whose JSON text exists already (the bulk downloads)
HttpResponse opt_text(std::optional<std::string>&& text) {
  if (!text) return not_found_resource();
  HttpResponse r;
  r.status = 200;
  r.content_type = "application/json";
  r.body = std::move(*text);
  return r;
}
template <class T>
HttpResponse vec_json(const std::vector<T>& v) {
  json::Value a = json::Value::array();
  for (auto& x : v) a.push(wire::to_json(x));
  return json_resp(a);
}
template <class T>
T body_as(const HttpRequest& req) {
  if (req.body.empty()) throw SdaError::invalid("Expected a body");
  try {
    return wire::decode<T>(req.body);
  } catch (const SdaError& e) {
    throw SdaError::invalid(e.what());
  }
}

}  // namespace

Agent SdaHttpHandler::caller(const HttpRequest& req) {
  return svc_->server().check_auth_token(parse_basic_auth(req.header("authorization")));
}

HttpResponse SdaHttpHandler::handle(const HttpRequest& req) {
  HttpResponse resp;
  try {
    auto seg = split(req.path, '/');  // "", "v1", ...
    if (!seg.empty() && seg[0].empty()) seg.erase(seg.begin());
    while (!seg.empty() && seg.back().empty()) seg.pop_back();
    const std::string& m = req.method;
    const size_t n = seg.size();
    auto is = [&](std::initializer_list<const char*> lits) {
      if (n != lits.size()) return false;
      size_t i = 0;
      for (const char* l : lits) {
        if (std::string(l) != "*" && seg[i] != l) return false;
        ++i;
      }
      return true;
    };
    if (n == 0 || seg[0] != "v1") {
      resp = empty(404);
    } else if (m == "GET" && is({"v1", "ping"})) {
      resp = json_resp(wire::to_json(svc_->ping()));
    } else if (m == "POST" && is({"v1", "agents", "me"})) {
      AuthToken auth = parse_basic_auth(req.header("authorization"));
      Agent agent = body_as<Agent>(req);
      if (agent.id != auth.id) {
        resp = empty(400);
        resp.body = "inconsistent agent ids";
      } else {
        // trust on first use; never let a second registration steal the token
        auto prev = svc_->server().stores().auth_tokens->get_auth_token(auth.id);
        if (prev && !(*prev == auth)) throw SdaError::invalid_credentials();
        svc_->create_agent(agent, agent);
        svc_->server().upsert_auth_token(auth);
        resp = empty(201);
      }
    } else if (m == "POST" && is({"v1", "agents", "me", "profile"})) {
      svc_->upsert_profile(caller(req), body_as<Profile>(req));
      resp = empty(201);
    } else if (m == "POST" && is({"v1", "agents", "me", "keys"})) {
      svc_->create_encryption_key(caller(req), body_as<SignedEncryptionKey>(req));
      resp = empty(201);
    } else if (m == "GET" && is({"v1", "agents", "any", "keys", "*"})) {
      resp = opt_json(svc_->get_encryption_key(caller(req), EncryptionKeyId::parse(seg[4])));
    } else if (m == "GET" && is({"v1", "agents", "*", "profile"})) {
      resp = opt_json(svc_->get_profile(caller(req), AgentId::parse(seg[2])));
    } else if (m == "GET" && is({"v1", "agents", "*"})) {
      resp = opt_json(svc_->get_agent(caller(req), AgentId::parse(seg[2])));
    } else if (m == "POST" && is({"v1", "aggregations"})) {
      svc_->create_aggregation(caller(req), body_as<Aggregation>(req));
      resp = empty(201);
    } else if (m == "GET" && is({"v1", "aggregations"})) {
      std::optional<std::string> title;
      std::optional<AgentId> recipient;
      if (req.query.count("title")) title = req.query.at("title");
      if (req.query.count("recipient")) recipient = AgentId::parse(req.query.at("recipient"));
      resp = vec_json(svc_->list_aggregations(caller(req), title, recipient));
    } else if (m == "POST" && is({"v1", "aggregations", "participations"})) {
      svc_->create_participation(caller(req), body_as<Participation>(req));
      resp = empty(201);
    } else if (m == "POST" && is({"v1", "aggregations", "implied", "committee"})) {
      svc_->create_committee(caller(req), body_as<Committee>(req));
      resp = empty(201);
    } else if (m == "POST" && is({"v1", "aggregations", "implied", "snapshot"})) {
      svc_->create_snapshot(caller(req), body_as<Snapshot>(req));
      resp = empty(201);
    } else if (m == "GET" && is({"v1", "aggregations", "any", "jobs"})) {
      Agent c = caller(req);
      resp = opt_text(svc_->get_clerking_job_json(c, c.id));
    } else if (m == "POST" && is({"v1", "aggregations", "implied", "jobs", "*", "result"})) {
      svc_->create_clerking_result(caller(req), body_as<ClerkingResult>(req));
      resp = empty(201);
    } else if (m == "GET" && is({"v1", "aggregations", "*", "committee", "suggestions"})) {
      resp = vec_json(svc_->suggest_committee(caller(req), AggregationId::parse(seg[2])));
    } else if (m == "GET" && is({"v1", "aggregations", "*", "committee"})) {
      resp = opt_json(svc_->get_committee(caller(req), AggregationId::parse(seg[2])));
    } else if (m == "GET" && is({"v1", "aggregations", "*", "status"})) {
      resp = opt_json(svc_->get_aggregation_status(caller(req), AggregationId::parse(seg[2])));
    } else if (m == "GET" && is({"v1", "aggregations", "*", "snapshots", "*", "result"})) {
      resp = opt_text(svc_->get_snapshot_result_json(caller(req), AggregationId::parse(seg[2]),
                                                     SnapshotId::parse(seg[4])));
    } else if (m == "GET" && is({"v1", "aggregations", "*"})) {
      resp = opt_json(svc_->get_aggregation(caller(req), AggregationId::parse(seg[2])));
    } else if (m == "DELETE" && is({"v1", "aggregations", "*"})) {
      svc_->delete_aggregation(caller(req), AggregationId::parse(seg[2]));
      resp = empty(200);
    } else {
      log_error("Route not found: " + m + " " + req.target);
      resp = empty(404);
    }
    log_info(m + " " + req.target + " (" + std::to_string(resp.status) + ")");
  } catch (const SdaError& e) {
    int code = 500;
    switch (e.kind()) {
      case ErrorKind::InvalidCredentials: code = 401; break;
      case ErrorKind::PermissionDenied: code = 403; break;
      case ErrorKind::Invalid: code = 400; break;
      default:
        // unparseable ids in the path are client errors
        code = std::string(e.what()).rfind("unparseable uuid", 0) == 0 ? 400 : 500;
    }
    log_error(req.method + " " + req.target + " " + e.what() + " (" + std::to_string(code) + ")");
    resp = empty(code);
    resp.content_type = "text/plain; charset=utf-8";
    resp.body = e.what();
  }
  return resp;
}

// ---- REST client ------------------------------------------------------------------
SdaHttpClient::SdaHttpClient(const std::string& server_root, StorePtr token_store)
    : tokens_(std::move(token_store)) {
  std::string r = server_root;
  if (r.rfind("http://", 0) != 0) throw SdaError("only http:// server roots are supported: " + r);
  r = r.substr(7);
  auto slash = r.find('/');
  std::string hostport = slash == std::string::npos ? r : r.substr(0, slash);
  prefix_ = slash == std::string::npos ? "" : r.substr(slash);
  while (!prefix_.empty() && prefix_.back() == '/') prefix_.pop_back();
  auto colon = hostport.rfind(':');
  host_ = colon == std::string::npos ? hostport : hostport.substr(0, colon);
  port_ = colon == std::string::npos ? 80 : std::stoi(hostport.substr(colon + 1));
}

SdaHttpClient::Reply SdaHttpClient::request(const std::string& method, const std::string& path,
                                            const Agent* caller, const std::string* json_body) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  std::string host = host_ == "localhost" ? "127.0.0.1" : host_;
  if (::getaddrinfo(host.c_str(), std::to_string(port_).c_str(), &hints, &res) != 0 || !res)
    throw SdaError("HTTP/REST error: cannot resolve " + host_);
  int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0 || ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    ::freeaddrinfo(res);
    if (fd >= 0) ::close(fd);
    throw SdaError("HTTP/REST error: cannot connect to " + host_ + ":" + std::to_string(port_));
  }
  ::freeaddrinfo(res);
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  std::ostringstream out;
  out << method << " " << prefix_ << path << " HTTP/1.1\r\nHost: " << host_ << ":" << port_
      << "\r\nUser-Agent: SDA CLI client\r\nConnection: close\r\n";
  if (caller) {
    std::string cred = caller->id.str() + ":" + tokens_->auth_token();
    out << "Authorization: Basic "
        << base64_encode(reinterpret_cast<const uint8_t*>(cred.data()), cred.size()) << "\r\n";
  }
  if (json_body) out << "Content-Type: application/json\r\nContent-Length: " << json_body->size() << "\r\n";
  else out << "Content-Length: 0\r\n";
  out << "\r\n";
  std::string head = out.str();
  bool ok = send_all(fd, head.data(), head.size()) &&
            (!json_body || send_all(fd, json_body->data(), json_body->size()));
  Reply rep;
  std::string buf, rhead;
  if (!ok || read_message(fd, buf, rhead, rep.body, true, (size_t)8 << 30) != ReadStatus::Ok) {
    ::close(fd);
    throw SdaError("HTTP/REST error: connection failed");
  }
  ::close(fd);
  auto lines = split(rhead, '\n');
  auto sl = split(trim(lines[0]), ' ');
  if (sl.size() < 2) throw SdaError("HTTP/REST error: bad status line");
  rep.status = std::stoi(sl[1]);
  for (size_t i = 1; i < lines.size(); ++i) {
    auto c = lines[i].find(':');
    if (c != std::string::npos) rep.headers[lower(trim(lines[i].substr(0, c)))] = trim(lines[i].substr(c + 1));
  }
  return rep;
}

std::optional<json::Value> SdaHttpClient::call(const std::string& method, const std::string& path,
                                               const Agent* caller, const std::string* body) {
  auto text = call_text(method, path, caller, body);
  if (!text) return std::nullopt;
  return json::Value::parse(*text);
}

std::optional<std::string> SdaHttpClient::call_text(const std::string& method, const std::string& path,
                                                    const Agent* caller, const std::string* body) {
  Reply r = request(method, path, caller, body);
  switch (r.status) {
    case 200:
    case 201:
      if (r.body.empty()) return std::nullopt;
      return std::move(r.body);
    case 404:
      if (r.headers.count("resource-not-found")) return std::nullopt;
      throw SdaError("HTTP/REST route not found");
    case 401: throw SdaError::invalid_credentials();
    case 403: throw SdaError::permission_denied();
    case 400: throw SdaError::invalid(r.body);
    default: throw SdaError("HTTP/REST error: " + std::to_string(r.status) + " " + r.body);
  }
}

namespace {
template <class T>
std::optional<T> opt_from(const std::optional<json::Value>& v) {
  if (!v) return std::nullopt;
  return wire::from_json<T>(*v);
}
template <class T>
T required(const std::optional<json::Value>& v) {
  if (!v) throw SdaError("Missing response payload");
  return wire::from_json<T>(*v);
}
template <class T>
std::vector<T> required_vec(const std::optional<json::Value>& v) {
  if (!v) throw SdaError("Missing response payload");
  std::vector<T> out;
  for (auto& x : v->as_array()) out.push_back(wire::from_json<T>(x));
  return out;
}
void no_payload(const std::optional<json::Value>& v) {
  if (v) throw SdaError("Extra response payload");
}
template <class T>
std::vector<T> ids_from(const std::optional<json::Value>& v) {
  if (!v) throw SdaError("Missing response payload");
  std::vector<T> out;
  for (auto& x : v->as_array()) out.push_back(T::parse(x.as_string()));
  return out;
}
}  // namespace

Pong SdaHttpClient::ping() { return required<Pong>(call("GET", "/v1/ping", nullptr, nullptr)); }
void SdaHttpClient::create_agent(const Agent& c, const Agent& a) {
  std::string b = wire::encode(a);
  no_payload(call("POST", "/v1/agents/me", &c, &b));
}
std::optional<Agent> SdaHttpClient::get_agent(const Agent& c, const AgentId& a) {
  return opt_from<Agent>(call("GET", "/v1/agents/" + a.str(), &c, nullptr));
}
void SdaHttpClient::upsert_profile(const Agent& c, const Profile& p) {
  std::string b = wire::encode(p);
  no_payload(call("POST", "/v1/agents/me/profile", &c, &b));
}
std::optional<Profile> SdaHttpClient::get_profile(const Agent& c, const AgentId& o) {
  return opt_from<Profile>(call("GET", "/v1/agents/" + o.str() + "/profile", &c, nullptr));
}
void SdaHttpClient::create_encryption_key(const Agent& c, const SignedEncryptionKey& k) {
  std::string b = wire::encode(k);
  no_payload(call("POST", "/v1/agents/me/keys", &c, &b));
}
std::optional<SignedEncryptionKey> SdaHttpClient::get_encryption_key(const Agent& c, const EncryptionKeyId& k) {
  return opt_from<SignedEncryptionKey>(call("GET", "/v1/agents/any/keys/" + k.str(), &c, nullptr));
}
std::vector<AggregationId> SdaHttpClient::list_aggregations(const Agent& c, const std::optional<std::string>& f,
                                                            const std::optional<AgentId>& r) {
  // the reference dropped the /v1 prefix here (client-http/src/client.rs:245-247)
  std::string path = "/v1/aggregations";
  std::string sep = "?";
  if (f) { path += sep + "title=" + url_encode(*f); sep = "&"; }
  if (r) path += sep + "recipient=" + r->str();
  return ids_from<AggregationId>(call("GET", path, &c, nullptr));
}
std::optional<Aggregation> SdaHttpClient::get_aggregation(const Agent& c, const AggregationId& a) {
  return opt_from<Aggregation>(call("GET", "/v1/aggregations/" + a.str(), &c, nullptr));
}
std::optional<Committee> SdaHttpClient::get_committee(const Agent& c, const AggregationId& a) {
  return opt_from<Committee>(call("GET", "/v1/aggregations/" + a.str() + "/committee", &c, nullptr));
}
void SdaHttpClient::create_participation(const Agent& c, const Participation& p) {
  std::string b = wire::encode(p);
  no_payload(call("POST", "/v1/aggregations/participations", &c, &b));
}
std::optional<ClerkingJob> SdaHttpClient::get_clerking_job(const Agent& c, const AgentId&) {
  return opt_from<ClerkingJob>(call("GET", "/v1/aggregations/any/jobs", &c, nullptr));
}
std::optional<std::string> SdaHttpClient::get_clerking_job_json(const Agent& c, const AgentId&) {
  return call_text("GET", "/v1/aggregations/any/jobs", &c, nullptr);
}
std::optional<std::string> SdaHttpClient::get_snapshot_result_json(const Agent& c, const AggregationId& a,
                                                                   const SnapshotId& s) {
  auto text = call_text("GET", "/v1/aggregations/" + a.str() + "/snapshots/" + s.str() + "/result", &c, nullptr);
  if (!text) throw SdaError("Missing response payload");
  return text;
}
void SdaHttpClient::create_clerking_result(const Agent& c, const ClerkingResult& r) {
  std::string b = wire::encode(r);
  no_payload(call("POST", "/v1/aggregations/implied/jobs/" + r.job.str() + "/result", &c, &b));
}
void SdaHttpClient::create_aggregation(const Agent& c, const Aggregation& a) {
  std::string b = wire::encode(a);
  no_payload(call("POST", "/v1/aggregations", &c, &b));
}
void SdaHttpClient::delete_aggregation(const Agent& c, const AggregationId& a) {
  no_payload(call("DELETE", "/v1/aggregations/" + a.str(), &c, nullptr));
}
std::vector<ClerkCandidate> SdaHttpClient::suggest_committee(const Agent& c, const AggregationId& a) {
  return required_vec<ClerkCandidate>(
      call("GET", "/v1/aggregations/" + a.str() + "/committee/suggestions", &c, nullptr));
}
void SdaHttpClient::create_committee(const Agent& c, const Committee& cm) {
  std::string b = wire::encode(cm);
  no_payload(call("POST", "/v1/aggregations/implied/committee", &c, &b));
}
std::optional<AggregationStatus> SdaHttpClient::get_aggregation_status(const Agent& c, const AggregationId& a) {
  return opt_from<AggregationStatus>(call("GET", "/v1/aggregations/" + a.str() + "/status", &c, nullptr));
}
void SdaHttpClient::create_snapshot(const Agent& c, const Snapshot& s) {
  std::string b = wire::encode(s);
  no_payload(call("POST", "/v1/aggregations/implied/snapshot", &c, &b));
}
std::optional<SnapshotResult> SdaHttpClient::get_snapshot_result(const Agent& c, const AggregationId& a,
                                                                 const SnapshotId& s) {
  return required<SnapshotResult>(
      call("GET", "/v1/aggregations/" + a.str() + "/snapshots/" + s.str() + "/result", &c, nullptr));
}

}  // namespace sda
