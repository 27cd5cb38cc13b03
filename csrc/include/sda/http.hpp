// HTTP/1.1 transport for SDA (reference server-http/src/lib.rs, client-http/src/*).
//
// Server: POSIX sockets, an accept thread and a worker pool; routes and status
// semantics of the reference REST API (server-http/src/lib.rs routes): JSON bodies, Basic auth
// `agent_id:token` with trust-on-first-use at POST /v1/agents/me, 404 +
// `Resource-not-found: true` for a missing resource, a bare 404 for an unknown
// route, 401 / 403 / 400 / 500 with a text body for errors.
// Client: `SdaHttpClient` implements SdaService over REST (the reference's
// central seam), User-Agent "SDA CLI client".
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "sda/client.hpp"
#include "sda/server.hpp"

namespace sda {

struct HttpRequest {
  std::string method;
  std::string target;  // raw path + query
  std::string path;
  std::map<std::string, std::string> query;
  std::map<std::string, std::string> headers;  // lower-case names
  std::string body;
  std::string header(const std::string& lower_name) const;
};

struct HttpResponse {
  int status = 200;
  std::string content_type;
  std::string body;
  std::vector<std::pair<std::string, std::string>> headers;
};

std::string url_decode(const std::string& s);
std::string url_encode(const std::string& s);

class HttpServer {
 public:
  using Handler = std::function<HttpResponse(const HttpRequest&)>;
  HttpServer(Handler handler, int threads = 8);
  ~HttpServer();
  // "127.0.0.1:8888" ; port 0 = ephemeral. Returns the bound port.
  int start(const std::string& bind);
  void stop();
  int port() const { return port_; }
  void serve_forever();  // block until stop()
  // Largest request body accepted (checked before the body is buffered; 413
  // beyond it). Default 256 MiB: a participation for a 1M-dimension aggregation
  // with 8 clerks is ~30 MB of base64.
  void set_max_body(size_t bytes) { max_body_ = bytes; }

 private:
  void accept_loop();
  void worker_loop();
  void handle_conn(int fd);
  Handler handler_;
  int threads_;
  size_t max_body_ = (size_t)256 << 20;
  int listen_fd_ = -1;
  int port_ = 0;
  std::atomic<bool> running_{false};
  std::thread acceptor_;
  std::vector<std::thread> workers_;
  struct Queue;
  std::unique_ptr<Queue> q_;
};

// The SDA REST router over an in-process server (server-http/src/lib.rs:131-296).
class SdaHttpHandler {
 public:
  explicit SdaHttpHandler(std::shared_ptr<SdaServerService> service) : svc_(std::move(service)) {}
  HttpResponse handle(const HttpRequest& req);

 private:
  Agent caller(const HttpRequest& req);
  std::shared_ptr<SdaServerService> svc_;
};

// Parse `Authorization: Basic base64(agent_id:token)` (server-http/src/lib.rs:298-315).
AuthToken parse_basic_auth(const std::string& header_value);

class SdaHttpClient : public SdaService {
 public:
  SdaHttpClient(const std::string& server_root, StorePtr token_store);

  Pong ping() override;
  void create_agent(const Agent& caller, const Agent& agent) override;
  std::optional<Agent> get_agent(const Agent& caller, const AgentId& agent) override;
  void upsert_profile(const Agent& caller, const Profile& profile) override;
  std::optional<Profile> get_profile(const Agent& caller, const AgentId& owner) override;
  void create_encryption_key(const Agent& caller, const SignedEncryptionKey& key) override;
  std::optional<SignedEncryptionKey> get_encryption_key(const Agent& caller,
                                                        const EncryptionKeyId& key) override;
  std::vector<AggregationId> list_aggregations(const Agent& caller,
                                               const std::optional<std::string>& filter,
                                               const std::optional<AgentId>& recipient) override;
  std::optional<Aggregation> get_aggregation(const Agent& caller, const AggregationId& a) override;
  std::optional<Committee> get_committee(const Agent& caller, const AggregationId& a) override;
  void create_participation(const Agent& caller, const Participation& p) override;
  std::optional<ClerkingJob> get_clerking_job(const Agent& caller, const AgentId& clerk) override;
  void create_clerking_result(const Agent& caller, const ClerkingResult& r) override;
  void create_aggregation(const Agent& caller, const Aggregation& a) override;
  void delete_aggregation(const Agent& caller, const AggregationId& a) override;
  std::vector<ClerkCandidate> suggest_committee(const Agent& caller, const AggregationId& a) override;
  void create_committee(const Agent& caller, const Committee& c) override;
  std::optional<AggregationStatus> get_aggregation_status(const Agent& caller,
                                                          const AggregationId& a) override;
  void create_snapshot(const Agent& caller, const Snapshot& s) override;
  std::optional<SnapshotResult> get_snapshot_result(const Agent& caller, const AggregationId& a,
                                                    const SnapshotId& s) override;
  // the bulk downloads as received (no JSON tree is built)
  std::optional<std::string> get_clerking_job_json(const Agent& caller, const AgentId& clerk) override;
  std::optional<std::string> get_snapshot_result_json(const Agent& caller, const AggregationId& a,
                                                      const SnapshotId& s) override;

  struct Reply {
    int status = 0;
    std::map<std::string, std::string> headers;
    std::string body;
  };
  Reply request(const std::string& method, const std::string& path, const Agent* caller,
                const std::string* json_body);

 private:
  // process(): status -> Some(json) / None / typed error (client-http/src/client.rs:43-102)
  std::optional<json::Value> call(const std::string& method, const std::string& path,
                                  const Agent* caller, const std::string* body);
  std::optional<std::string> call_text(const std::string& method, const std::string& path,
                                  const Agent* caller, const std::string* body);
  std::string host_;
  int port_ = 80;
  std::string prefix_;
  StorePtr tokens_;
};

}  // namespace sda
