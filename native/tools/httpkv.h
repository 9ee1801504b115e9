// Minimal blocking HTTP/1.1 client for the control-plane KV store (unique-id rendezvous of
// multi-process RCCL jobs). Supports http://host:port/path only; one request per connection.
#pragma once

#include <arpa/inet.h>
#include <netdb.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>

namespace tk8s {

struct HttpResponse {
  int status = 0;
  std::string body;
};

// The bearer token for the control plane (it answers no anonymous KV request): TK8S_KV_TOKEN,
// else the pod's ServiceAccount token file (process pods: TK8S_SERVICEACCOUNT_TOKEN_FILE; image
// pods: the Kubernetes mount path). Empty when there is none.
inline std::string kv_bearer() {
  if (const char* t = std::getenv("TK8S_KV_TOKEN"); t && *t) return t;
  const char* named = std::getenv("TK8S_SERVICEACCOUNT_TOKEN_FILE");
  for (const char* path : {named, "/var/run/secrets/kubernetes.io/serviceaccount/token"}) {
    if (!path || !*path) continue;
    std::ifstream f(path);
    std::string tok;
    if (f >> tok && !tok.empty()) return tok;
  }
  return {};
}

inline bool http_request(const std::string& method, const std::string& url, const std::string& body,
                         HttpResponse* out, int timeout_s = 60) {
  if (url.rfind("http://", 0) != 0) return false;
  const std::string rest = url.substr(7);
  const auto slash = rest.find('/');
  const std::string hostport = rest.substr(0, slash);
  const std::string path = slash == std::string::npos ? "/" : rest.substr(slash);
  const auto colon = hostport.rfind(':');
  const std::string host = hostport.substr(0, colon);
  const std::string port = colon == std::string::npos ? "80" : hostport.substr(colon + 1);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) return false;
  const int fd = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0) {
    freeaddrinfo(res);
    return false;
  }
  timeval tv{timeout_s, 0};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  const bool connected = connect(fd, res->ai_addr, res->ai_addrlen) == 0;
  freeaddrinfo(res);
  if (!connected) {
    close(fd);
    return false;
  }
  const std::string bearer = kv_bearer();
  const std::string auth = bearer.empty() ? std::string() : "Authorization: Bearer " + bearer + "\r\n";
  std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + hostport +
                    "\r\nConnection: close\r\nContent-Type: text/plain\r\n" + auth + "Content-Length: " +
                    std::to_string(body.size()) + "\r\n\r\n" + body;
  size_t sent = 0;
  while (sent < req.size()) {
    const ssize_t k = send(fd, req.data() + sent, req.size() - sent, 0);
    if (k <= 0) {
      close(fd);
      return false;
    }
    sent += static_cast<size_t>(k);
  }
  std::string resp;
  char buf[4096];
  for (;;) {
    const ssize_t k = recv(fd, buf, sizeof buf, 0);
    if (k <= 0) break;
    resp.append(buf, static_cast<size_t>(k));
  }
  close(fd);
  const auto sp = resp.find(' ');
  const auto hdr_end = resp.find("\r\n\r\n");
  if (sp == std::string::npos || hdr_end == std::string::npos) return false;
  out->status = std::atoi(resp.c_str() + sp + 1);
  out->body = resp.substr(hdr_end + 4);
  return true;
}

}  // namespace tk8s
