// sq_sockaddr.h -- sqobfs_addr <-> struct sockaddr (udp_batch.cpp, pconn.cpp).
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <string.h>
#include <sys/socket.h>

#include "sqobfs.h"

namespace sq {

inline void to_sockaddr(const sqobfs_addr &a, sockaddr_storage *ss, socklen_t *sl) {
  memset(ss, 0, sizeof *ss);
  if (a.family == AF_INET6) {
    auto *s6 = reinterpret_cast<sockaddr_in6 *>(ss);
    s6->sin6_family = AF_INET6;
    s6->sin6_port = htons(a.port);
    s6->sin6_scope_id = a.scope_id;
    memcpy(&s6->sin6_addr, a.addr, 16);
    *sl = sizeof(sockaddr_in6);
  } else {
    auto *s4 = reinterpret_cast<sockaddr_in *>(ss);
    s4->sin_family = AF_INET;
    s4->sin_port = htons(a.port);
    memcpy(&s4->sin_addr, a.addr, 4);
    *sl = sizeof(sockaddr_in);
  }
}

inline void from_sockaddr(const sockaddr_storage &ss, sqobfs_addr *a) {
  memset(a, 0, sizeof *a);
  if (ss.ss_family == AF_INET6) {
    const auto *s6 = reinterpret_cast<const sockaddr_in6 *>(&ss);
    a->family = AF_INET6;
    a->port = ntohs(s6->sin6_port);
    a->scope_id = s6->sin6_scope_id;
    memcpy(a->addr, &s6->sin6_addr, 16);
  } else if (ss.ss_family == AF_INET) {
    const auto *s4 = reinterpret_cast<const sockaddr_in *>(&ss);
    a->family = AF_INET;
    a->port = ntohs(s4->sin_port);
    memcpy(a->addr, &s4->sin_addr, 4);
  }
}

}  // namespace sq
