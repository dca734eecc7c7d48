// refnet_layer.hpp -- test infrastructure for oracle/refnet/build.py's crc_src
// variant: the layer object the INTEGRATION.md edits call, force-included
// (g++ -include) into the reference's net_manager.cpp before its send_raw and
// receive_logic are rewritten to the INTEGRATION.md snippets.
//
// INTEGRATION.md makes the layer a net_manager member (m_crc_layer); the
// rewrite cannot add a member without editing the reference's header, so each
// net_manager gets its own lnl::crc32c_layer from this registry instead, keyed
// by the manager's address.  One receive thread per manager calls
// process_inbound_packet on its layer (as with a member); refnet_dropped()
// (refnet_wrap.cpp) sums the layers' drop counts.
#pragma once
#include <map>
#include <mutex>

#include "../../include/lnl_crc32c_layer.hpp"

inline std::mutex& refnet_layers_mu() {
    static std::mutex mu;
    return mu;
}
inline std::map<const void*, lnl::crc32c_layer*>& refnet_layers() {
    static std::map<const void*, lnl::crc32c_layer*> m;  // never freed: the driver reads the counts at exit
    return m;
}
inline lnl::crc32c_layer& refnet_crc_layer(const void* manager) {
    std::lock_guard<std::mutex> lk(refnet_layers_mu());
    lnl::crc32c_layer*& p = refnet_layers()[manager];
    if (!p) p = new lnl::crc32c_layer();
    return *p;
}
inline uint64_t refnet_layers_dropped() {
    std::lock_guard<std::mutex> lk(refnet_layers_mu());
    uint64_t d = 0;
    for (auto& kv : refnet_layers()) d += kv.second->dropped();
    return d;
}
