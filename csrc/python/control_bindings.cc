// pybind11 bindings, part 2: the control plane (`_sda_native.control`).
//
// Objects cross the boundary in their wire form (serde-compatible JSON text,
// protocol.hpp); the Python layer (`sda_amd.control`) turns them into dicts.
// Every potentially blocking call releases the GIL, so an in-process HTTP
// server, clerks on Python threads and a client can all run concurrently.
//
// Reference seams mirrored here: protocol/src/methods.rs (SdaService),
// server/src/lib.rs:34-45 (memory/JFS factories), server-store-mongodb
// (document store), server-http/src/lib.rs (REST server), client-http
// (REST client), client/src/lib.rs (SdaClient roles), client-store (stores).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sda/client.hpp"
#include "sda/http.hpp"
#include "sda/log.hpp"
#include "sda/server.hpp"

namespace py = pybind11;
using namespace sda;

namespace {

using GilRelease = py::call_guard<py::gil_scoped_release>;

template <class T>
T dec(const std::string& s) { return wire::decode<T>(s); }
template <class T>
std::string enc(const T& x) { return wire::encode(x); }
template <class T>
std::optional<std::string> enc_opt(const std::optional<T>& x) {
  if (!x) return std::nullopt;
  return wire::encode(*x);
}
template <class T>
std::vector<std::string> enc_vec(const std::vector<T>& xs) {
  std::vector<std::string> out;
  out.reserve(xs.size());
  for (const auto& x : xs) out.push_back(wire::encode(x));
  return out;
}
template <class Id>
std::vector<std::string> ids(const std::vector<Id>& xs) {
  std::vector<std::string> out;
  for (const auto& x : xs) out.push_back(x.str());
  return out;
}

// A running REST server over a service; stops on destruction.
struct HttpServerHandle {
  std::shared_ptr<SdaServerService> svc;
  std::shared_ptr<SdaHttpHandler> handler;
  std::unique_ptr<HttpServer> server;
  HttpServerHandle(std::shared_ptr<SdaServerService> s, int threads)
      : svc(std::move(s)), handler(std::make_shared<SdaHttpHandler>(svc)) {
    auto h = handler;
    server = std::make_unique<HttpServer>([h](const HttpRequest& r) { return h->handle(r); },
                                          threads);
  }
};

}  // namespace

void bind_control_plane(py::module_& m) {
  auto c = m.def_submodule("control", "SDA control plane: server, stores, REST, client roles");

  // error kinds (protocol/src/lib.rs:21-41)
  // leaked on purpose: no Python decref after interpreter finalisation
  static auto* base_exc = new py::exception<SdaError>(c, "SdaError");
  static auto* perm_exc = new py::exception<SdaError>(c, "PermissionDenied", base_exc->ptr());
  static auto* cred_exc = new py::exception<SdaError>(c, "InvalidCredentials", base_exc->ptr());
  static auto* inv_exc = new py::exception<SdaError>(c, "Invalid", base_exc->ptr());
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const SdaError& e) {
      switch (e.kind()) {
        case ErrorKind::PermissionDenied: py::set_error(*perm_exc, e.what()); break;
        case ErrorKind::InvalidCredentials: py::set_error(*cred_exc, e.what()); break;
        case ErrorKind::Invalid: py::set_error(*inv_exc, e.what()); break;
        default: py::set_error(*base_exc, e.what()); break;
      }
    }
  });

  c.def("set_log_level", &set_log_level, "slog levels: 1=critical .. 4=info .. 6=trace");
  c.def("log_level", &log_level);

  // ---- wire format --------------------------------------------------------
  c.def("canonicalize", [](const std::string& type, const std::string& text) -> std::string {
    // decode + re-encode: validates a wire object and yields the canonical text
#define SDA_WIRE(T) if (type == #T) return enc(dec<T>(text));
    SDA_WIRE(Agent) SDA_WIRE(Profile) SDA_WIRE(SignedEncryptionKey) SDA_WIRE(Aggregation)
    SDA_WIRE(ClerkCandidate) SDA_WIRE(Committee) SDA_WIRE(Participation) SDA_WIRE(Snapshot)
    SDA_WIRE(ClerkingJob) SDA_WIRE(ClerkingResult) SDA_WIRE(SnapshotStatus)
    SDA_WIRE(AggregationStatus) SDA_WIRE(SnapshotResult) SDA_WIRE(Pong) SDA_WIRE(AuthToken)
    SDA_WIRE(LinearMaskingScheme) SDA_WIRE(LinearSecretSharingScheme)
    SDA_WIRE(AdditiveEncryptionScheme) SDA_WIRE(Encryption) SDA_WIRE(EncryptionKey)
    SDA_WIRE(EncryptionKeypair) SDA_WIRE(SignatureKeypair)
#undef SDA_WIRE
    throw std::invalid_argument("unknown wire type " + type);
  });
  c.def("new_id", []() { return Uuid::random().str(); });
  c.def("base64_encode", [](py::bytes b) {
    std::string s = b;
    return base64_encode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  c.def("base64_decode", [](const std::string& s) {
    Bytes b = base64_decode(s);
    return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
  });

  // ---- service --------------------------------------------------------------
  py::class_<SdaService, ServicePtr>(c, "Service",
                                     "SdaService (methods.rs): objects as wire-JSON strings")
      .def("ping", [](SdaService& s) { return enc(s.ping()); }, GilRelease())
      .def("create_agent", [](SdaService& s, const std::string& caller, const std::string& a) {
        s.create_agent(dec<Agent>(caller), dec<Agent>(a));
      }, GilRelease())
      .def("get_agent", [](SdaService& s, const std::string& caller, const std::string& id) {
        return enc_opt(s.get_agent(dec<Agent>(caller), AgentId::parse(id)));
      }, GilRelease())
      .def("upsert_profile", [](SdaService& s, const std::string& caller, const std::string& p) {
        s.upsert_profile(dec<Agent>(caller), dec<Profile>(p));
      }, GilRelease())
      .def("get_profile", [](SdaService& s, const std::string& caller, const std::string& id) {
        return enc_opt(s.get_profile(dec<Agent>(caller), AgentId::parse(id)));
      }, GilRelease())
      .def("create_encryption_key", [](SdaService& s, const std::string& caller,
                                       const std::string& k) {
        s.create_encryption_key(dec<Agent>(caller), dec<SignedEncryptionKey>(k));
      }, GilRelease())
      .def("get_encryption_key", [](SdaService& s, const std::string& caller,
                                    const std::string& id) {
        return enc_opt(s.get_encryption_key(dec<Agent>(caller), EncryptionKeyId::parse(id)));
      }, GilRelease())
      .def("list_aggregations", [](SdaService& s, const std::string& caller,
                                   std::optional<std::string> filter,
                                   std::optional<std::string> recipient) {
        std::optional<AgentId> r;
        if (recipient) r = AgentId::parse(*recipient);
        return ids(s.list_aggregations(dec<Agent>(caller), filter, r));
      }, py::arg("caller"), py::arg("filter") = py::none(), py::arg("recipient") = py::none(),
         GilRelease())
      .def("get_aggregation", [](SdaService& s, const std::string& caller, const std::string& id) {
        return enc_opt(s.get_aggregation(dec<Agent>(caller), AggregationId::parse(id)));
      }, GilRelease())
      .def("get_committee", [](SdaService& s, const std::string& caller, const std::string& id) {
        return enc_opt(s.get_committee(dec<Agent>(caller), AggregationId::parse(id)));
      }, GilRelease())
      .def("create_participation", [](SdaService& s, const std::string& caller,
                                      const std::string& p) {
        s.create_participation(dec<Agent>(caller), dec<Participation>(p));
      }, GilRelease())
      .def("get_clerking_job", [](SdaService& s, const std::string& caller,
                                  const std::string& clerk) {
        return enc_opt(s.get_clerking_job(dec<Agent>(caller), AgentId::parse(clerk)));
      }, GilRelease())
      .def("create_clerking_result", [](SdaService& s, const std::string& caller,
                                        const std::string& r) {
        s.create_clerking_result(dec<Agent>(caller), dec<ClerkingResult>(r));
      }, GilRelease())
      .def("create_aggregation", [](SdaService& s, const std::string& caller,
                                    const std::string& a) {
        s.create_aggregation(dec<Agent>(caller), dec<Aggregation>(a));
      }, GilRelease())
      .def("delete_aggregation", [](SdaService& s, const std::string& caller,
                                    const std::string& id) {
        s.delete_aggregation(dec<Agent>(caller), AggregationId::parse(id));
      }, GilRelease())
      .def("suggest_committee", [](SdaService& s, const std::string& caller,
                                   const std::string& id) {
        return enc_vec(s.suggest_committee(dec<Agent>(caller), AggregationId::parse(id)));
      }, GilRelease())
      .def("create_committee", [](SdaService& s, const std::string& caller,
                                  const std::string& cm) {
        s.create_committee(dec<Agent>(caller), dec<Committee>(cm));
      }, GilRelease())
      .def("get_aggregation_status", [](SdaService& s, const std::string& caller,
                                        const std::string& id) {
        return enc_opt(s.get_aggregation_status(dec<Agent>(caller), AggregationId::parse(id)));
      }, GilRelease())
      .def("create_snapshot", [](SdaService& s, const std::string& caller,
                                 const std::string& snap) {
        s.create_snapshot(dec<Agent>(caller), dec<Snapshot>(snap));
      }, GilRelease())
      .def("get_snapshot_result", [](SdaService& s, const std::string& caller,
                                     const std::string& agg, const std::string& snap) {
        return enc_opt(s.get_snapshot_result(dec<Agent>(caller), AggregationId::parse(agg),
                                             SnapshotId::parse(snap)));
      }, GilRelease())
      // the bulk downloads as the response text (see SdaService)
      .def("get_clerking_job_json", [](SdaService& s, const std::string& caller,
                                       const std::string& clerk) {
        return s.get_clerking_job_json(dec<Agent>(caller), AgentId::parse(clerk));
      }, GilRelease())
      .def("get_snapshot_result_json", [](SdaService& s, const std::string& caller,
                                          const std::string& agg, const std::string& snap) {
        return s.get_snapshot_result_json(dec<Agent>(caller), AggregationId::parse(agg),
                                          SnapshotId::parse(snap));
      }, GilRelease());

  // in-process server: the service plus server-side helpers (auth tokens)
  py::class_<SdaServerService, SdaService, std::shared_ptr<SdaServerService>>(c, "ServerService")
      .def("upsert_auth_token", [](SdaServerService& s, const std::string& t) {
        s.server().upsert_auth_token(dec<AuthToken>(t));
      }, GilRelease())
      .def("check_auth_token", [](SdaServerService& s, const std::string& t) {
        return enc(s.server().check_auth_token(dec<AuthToken>(t)));
      }, GilRelease())
      .def("delete_auth_token", [](SdaServerService& s, const std::string& id) {
        s.server().delete_auth_token(AgentId::parse(id));
      }, GilRelease())
      .def("poll_clerking_job", [](SdaServerService& s, const std::string& clerk) {
        return enc_opt(s.server().poll_clerking_job(AgentId::parse(clerk)));
      }, GilRelease());

  c.def("memory_server", &new_memory_server, "in-memory stores (server/src/lib.rs:34-37)");
  c.def("jfs_server", &new_jfs_server, py::arg("dir"),
        "JSON-file stores in a directory tree (server/src/lib.rs:39-45)");
  c.def("document_server", &new_document_server, py::arg("dir"),
        "document-collection stores (the Mongo data model, server-store-mongodb)");

  // ---- REST ----------------------------------------------------------------
  py::class_<HttpServerHandle, std::shared_ptr<HttpServerHandle>>(c, "HttpServer")
      .def(py::init<std::shared_ptr<SdaServerService>, int>(), py::arg("service"),
           py::arg("threads") = 8)
      .def("start", [](HttpServerHandle& h, const std::string& bind) {
        return h.server->start(bind);
      }, py::arg("bind") = "127.0.0.1:0", GilRelease())
      .def("stop", [](HttpServerHandle& h) { h.server->stop(); }, GilRelease())
      .def("serve_forever", [](HttpServerHandle& h) { h.server->serve_forever(); }, GilRelease())
      .def_property_readonly("port", [](HttpServerHandle& h) { return h.server->port(); });
  c.def("http_handle", [](std::shared_ptr<SdaServerService> svc, const std::string& method,
                          const std::string& target, std::map<std::string, std::string> headers,
                          const std::string& body) {
    // dispatch one request through the router without a socket (route tests)
    HttpRequest r;
    r.method = method;
    r.target = target;
    auto q = target.find('?');
    r.path = url_decode(target.substr(0, q));
    if (q != std::string::npos) {
      std::string qs = target.substr(q + 1);
      size_t i = 0;
      while (i <= qs.size()) {
        size_t amp = qs.find('&', i);
        if (amp == std::string::npos) amp = qs.size();
        std::string kv = qs.substr(i, amp - i);
        auto eq = kv.find('=');
        if (!kv.empty())
          r.query[url_decode(kv.substr(0, eq))] =
              eq == std::string::npos ? "" : url_decode(kv.substr(eq + 1));
        i = amp + 1;
      }
    }
    for (auto& [k, v] : headers) {
      std::string lk = k;
      for (auto& ch : lk) ch = (char)std::tolower((unsigned char)ch);
      r.headers[lk] = v;
    }
    r.body = body;
    SdaHttpHandler h(svc);
    HttpResponse resp;
    {
      py::gil_scoped_release nogil;
      resp = h.handle(r);
    }
    std::map<std::string, std::string> hs;
    for (auto& [k, v] : resp.headers) hs[k] = v;
    return py::make_tuple(resp.status, hs, py::bytes(resp.body));
  });
  c.def("parse_basic_auth", [](const std::string& v) { return enc(parse_basic_auth(v)); });

  // ---- client stores --------------------------------------------------------
  py::class_<Store, StorePtr>(c, "Store")
      .def("put", [](Store& s, const std::string& id, const std::string& v) {
        s.put_json(id, json::Value::parse(v));
      })
      .def("get", [](Store& s, const std::string& id) -> std::optional<std::string> {
        auto v = s.get_json(id);
        if (!v) return std::nullopt;
        return v->dump();
      })
      .def("define_alias", &Store::define_alias)
      .def("resolve_alias", &Store::resolve_alias)
      .def("auth_token", &Store::auth_token);
  py::class_<FileStore, Store, std::shared_ptr<FileStore>>(c, "FileStore")
      .def(py::init<const std::string&>(), py::arg("dir"))
      .def_property_readonly("dir", &FileStore::dir);
  py::class_<MemoryStore, Store, std::shared_ptr<MemoryStore>>(c, "MemoryStore").def(py::init<>());

  c.def("http_client", [](const std::string& root, StorePtr tokens) -> ServicePtr {
    return std::make_shared<SdaHttpClient>(root, std::move(tokens));
  }, py::arg("server_root"), py::arg("token_store"),
     "SdaService over REST (client-http/src/client.rs)");

  // ---- client-side crypto engines (client/src/crypto/*) ---------------------
  c.def("mask_secrets", [](const std::string& scheme, const std::vector<int64_t>& secrets) {
    auto r = mask_secrets(dec<LinearMaskingScheme>(scheme), secrets);
    return py::make_tuple(r.mask, r.masked_secrets);
  });
  c.def("combine_masks", [](const std::string& scheme,
                            const std::vector<std::vector<int64_t>>& masks) {
    return combine_masks(dec<LinearMaskingScheme>(scheme), masks);
  });
  c.def("unmask", [](const std::string& scheme, const std::vector<int64_t>& mask,
                     const std::vector<int64_t>& masked) {
    return unmask(dec<LinearMaskingScheme>(scheme), mask, masked);
  });
  c.def("generate_shares", [](const std::string& scheme, const std::vector<int64_t>& secrets) {
    return generate_shares(dec<LinearSecretSharingScheme>(scheme), secrets);
  });
  c.def("combine_shares", [](const std::string& scheme,
                             const std::vector<std::vector<int64_t>>& shares) {
    return combine_shares(dec<LinearSecretSharingScheme>(scheme), shares);
  });
  c.def("reconstruct_secrets", [](const std::string& scheme, uint64_t dimension,
                                  const std::vector<std::pair<size_t, std::vector<int64_t>>>& ix) {
    return reconstruct_secrets(dec<LinearSecretSharingScheme>(scheme), dimension, ix);
  });
  c.def("varint_encode", [](const std::vector<int64_t>& v) {
    Bytes b = varint_encode(v);
    return py::bytes(reinterpret_cast<const char*>(b.data()), b.size());
  });
  c.def("varint_decode", [](py::bytes b) {
    std::string s = b;
    return varint_decode(Bytes(s.begin(), s.end()));
  });
  c.def("encrypt_shares", [](const std::string& ek, const std::vector<int64_t>& shares) {
    return enc(encrypt_shares(dec<EncryptionKey>(ek), shares));
  }, GilRelease());
  c.def("decrypt_shares", [](const std::string& kp, const std::string& e) {
    return decrypt_shares(dec<EncryptionKeypair>(kp), dec<Encryption>(e));
  }, GilRelease());

  // ---- zero-copy views of the bulk downloads (wire_views.cc) --------------------
  c.def("scan_clerking_job", [](const std::string& text) -> py::object {
    auto v = wire::scan_clerking_job(text);
    if (!v) return py::none();
    std::vector<std::pair<size_t, size_t>> spans;
    for (auto& s : v->boxes) spans.emplace_back(s.off, s.len);
    return py::make_tuple(enc(v->head), spans);
  });
  c.def("scan_snapshot_result", [](const std::string& text) -> py::object {
    auto v = wire::scan_snapshot_result(text);
    if (!v) return py::none();
    std::vector<std::tuple<std::string, std::string, size_t, size_t>> results;
    for (auto& r : v->results) results.emplace_back(r.job.str(), r.clerk.str(), r.box.off, r.box.len);
    std::vector<std::pair<size_t, size_t>> masks;
    for (auto& s : v->masks) masks.emplace_back(s.off, s.len);
    return py::make_tuple(v->snapshot.str(), v->number_of_participations, results, v->has_masks, masks);
  });

  // ---- client roles (client/src/lib.rs + participate/clerk/receive/maintenance)
  py::class_<SdaClient, std::shared_ptr<SdaClient>>(c, "Client")
      .def(py::init([](const std::string& agent, StorePtr ks, ServicePtr svc) {
        return std::make_shared<SdaClient>(dec<Agent>(agent), std::move(ks), std::move(svc));
      }), py::arg("agent"), py::arg("keystore"), py::arg("service"))
      .def_static("new_agent", [](StorePtr ks) { return enc(SdaClient::new_agent(*ks)); })
      .def_property_readonly("agent", [](SdaClient& c) { return enc(c.agent()); })
      .def_property_readonly("service", [](SdaClient& c) { return c.service_ptr(); })
      .def("upload_agent", &SdaClient::upload_agent, GilRelease())
      .def("new_encryption_key", [](SdaClient& c) { return c.new_encryption_key().str(); },
           GilRelease())
      .def("upload_encryption_key", [](SdaClient& c, const std::string& id) {
        c.upload_encryption_key(EncryptionKeyId::parse(id));
      }, GilRelease())
      .def("sign_export", [](SdaClient& c, const std::string& id) {
        return enc_opt(c.sign_export(EncryptionKeyId::parse(id)));
      }, GilRelease())
      .def("new_participation", [](SdaClient& c, const std::vector<int64_t>& input,
                                   const std::string& agg) {
        return enc(c.new_participation(input, AggregationId::parse(agg)));
      }, GilRelease())
      .def("upload_participation", [](SdaClient& c, const std::string& p) {
        c.upload_participation(dec<Participation>(p));
      }, GilRelease())
      .def("participate", [](SdaClient& c, const std::vector<int64_t>& input,
                             const std::string& agg) {
        c.participate(input, AggregationId::parse(agg));
      }, GilRelease())
      .def("new_participations", [](SdaClient& c, const std::vector<std::vector<int64_t>>& inputs,
                                    const std::string& agg) {
        std::vector<std::string> out;
        for (auto& p : c.new_participations(inputs, AggregationId::parse(agg))) out.push_back(enc(p));
        return out;
      }, GilRelease())
      .def("participate_many", [](SdaClient& c, const std::vector<std::vector<int64_t>>& inputs,
                                  const std::string& agg) {
        c.participate_many(inputs, AggregationId::parse(agg));
      }, GilRelease())
      // GPU backend of the roles (libsda_device.so, loaded on demand)
      .def("use_device", [](SdaClient& c, const std::string& path, int index) {
        c.set_device_backend(load_device_backend(path, index));
        return c.device_backend()->describe();
      }, py::arg("path") = "", py::arg("index") = 0, GilRelease())
      .def("use_host", [](SdaClient& c) { c.set_device_backend(nullptr); })
      .def_property_readonly("device", [](SdaClient& c) -> std::optional<std::string> {
        if (!c.device_backend()) return std::nullopt;
        return c.device_backend()->describe();
      })
      .def("device_timings", [](SdaClient& c) {
        return c.device_backend() ? c.device_backend()->last_timings()
                                  : std::map<std::string, double>{};
      })
      .def("role_timings", &SdaClient::role_timings)
      .def("participate_array", [](SdaClient& c, py::array_t<int64_t, py::array::c_style | py::array::forcecast> a,
                                   const std::string& agg) {
        if (a.ndim() != 2) throw std::invalid_argument("participate_array: expected a [P][D] array");
        std::vector<std::vector<int64_t>> inputs(a.shape(0));
        const int64_t* p = a.data();
        for (ssize_t i = 0; i < a.shape(0); ++i) inputs[i].assign(p + i * a.shape(1), p + (i + 1) * a.shape(1));
        py::gil_scoped_release nogil;
        c.participate_many(inputs, AggregationId::parse(agg));
      })
      .def_static("device_unsupported", [](const std::string& agg) {
        return SdaClient::device_unsupported(dec<Aggregation>(agg));
      })
      .def("clerk_once", &SdaClient::clerk_once, GilRelease())
      .def("run_chores", &SdaClient::run_chores, py::arg("max_iterations") = -1, GilRelease())
      .def("process_clerking_job", [](SdaClient& c, const std::string& job) {
        return enc(c.process_clerking_job(dec<ClerkingJob>(job)));
      }, GilRelease())
      .def("upload_aggregation", [](SdaClient& c, const std::string& a) {
        c.upload_aggregation(dec<Aggregation>(a));
      }, GilRelease())
      .def("begin_aggregation", [](SdaClient& c, const std::string& a) {
        c.begin_aggregation(AggregationId::parse(a));
      }, GilRelease())
      .def("end_aggregation", [](SdaClient& c, const std::string& a) {
        c.end_aggregation(AggregationId::parse(a));
      }, GilRelease())
      .def("reveal_aggregation", [](SdaClient& c, const std::string& a) {
        RecipientOutput out;
        {
          py::gil_scoped_release nogil;
          out = c.reveal_aggregation(AggregationId::parse(a));
        }
        return py::make_tuple(out.modulus, out.values);
      });
}
