// `sdad` -- the SDA server daemon (reference server-cli/src/{lib.rs,bin/sdad.rs}).
//
//   sdad [-v...] (--jfs DIR | --document DIR | --memory) httpd [-b IP:PORT] [--threads N]
//
// Stores: `--jfs` is the reference's JSON-file layout; `--document` the
// document-collection store with the reference's MongoDB data model (no MongoDB
// server in this environment; `--mongo URL` is accepted and reported as
// unavailable); `--memory` keeps everything in RAM (tests, demos).
// SIGINT / SIGTERM stop the server cleanly.
#include <csignal>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "sda/http.hpp"
#include "sda/log.hpp"
#include "sda/server.hpp"

using namespace sda;

namespace {

volatile std::sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

[[noreturn]] void usage(const std::string& why = "") {
  if (!why.empty()) std::fprintf(stderr, "error: %s\n\n", why.c_str());
  std::fprintf(stderr,
               "usage: sdad [-v...] (--jfs DIR | --document DIR | --memory) httpd "
               "[-b IP:PORT] [--threads N] [--max-body-mb N]\n"
               "  httpd   run the REST server (default bind 127.0.0.1:8888)\n");
  std::exit(2);
}

}  // namespace

int main(int argc, char** argv) {
  std::string jfs, doc, mongo, bind = "127.0.0.1:8888", sub;
  bool memory = false;
  int verbose = 0, threads = 8;
  size_t max_body_mb = 256;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto val = [&](const char* what) -> std::string {
      if (i + 1 >= argc) usage(std::string(what) + " needs a value");
      return argv[++i];
    };
    if (s == "-h" || s == "--help") usage();
    else if (s == "--jfs") jfs = val("--jfs");
    else if (s == "--document" || s == "--doc") doc = val("--document");
    else if (s == "--mongo") mongo = val("--mongo");
    else if (s == "--mongo_dbname") (void)val("--mongo_dbname");
    else if (s == "--memory") memory = true;
    else if (s == "-b" || s == "--bind") bind = val("--bind");
    else if (s == "--threads") threads = std::stoi(val("--threads"));
    else if (s == "--max-body-mb") max_body_mb = std::stoul(val("--max-body-mb"));
    else if (s.size() > 1 && s[0] == '-' && s.find_first_not_of('v', 1) == std::string::npos)
      verbose += (int)s.size() - 1;
    else if (s == "--verbose") ++verbose;
    else if (sub.empty() && s[0] != '-') sub = s;
    else usage("unexpected argument " + s);
  }
  set_log_level(2 + verbose);  // errors by default, like the reference daemon
  try {
    std::shared_ptr<SdaServerService> svc;
    if (!mongo.empty())
      throw SdaError("no MongoDB in this build; use --document DIR (same data model)");
    if (!jfs.empty()) svc = new_jfs_server(jfs);
    else if (!doc.empty()) svc = new_document_server(doc);
    else if (memory) svc = new_memory_server();
    else throw SdaError("need a store configuration");
    if (sub != "httpd") throw SdaError("Unknown subcommand");
    auto handler = std::make_shared<SdaHttpHandler>(svc);
    HttpServer server([handler](const HttpRequest& r) { return handler->handle(r); }, threads);
    server.set_max_body(max_body_mb << 20);
    const int port = server.start(bind);
    log_info("Starting server on " + bind + " (port " + std::to_string(port) + ")");
    std::printf("listening on port %d\n", port);
    std::fflush(stdout);
    std::signal(SIGINT, on_signal);
    std::signal(SIGTERM, on_signal);
    while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    server.stop();
    return 0;
  } catch (const std::exception& e) {
    log_error(e.what());
    return 1;
  }
}
