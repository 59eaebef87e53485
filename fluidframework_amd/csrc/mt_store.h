/*
 * mt_store.h — column allocation for a batch of documents (host malloc or hipMalloc).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "mt_core.h"

namespace mt {

/* bytes of every column for `ndocs` documents with capacities k; fills c from `base` */
inline size_t layout(Cols& c, const Caps& k, int64_t ndocs, uint8_t* base) {
    size_t off = 0;
    auto take = [&](size_t bytes) -> uint8_t* {
        off = (off + 255) & ~(size_t)255;
        uint8_t* p = base ? base + off : nullptr;
        off += bytes;
        return p;
    };
    int64_t rows = (int64_t)k.ncap * MAXN * ndocs, nodes = (int64_t)k.ncap * ndocs;
    c.len = (int32_t*)take(4 * rows);
    c.seq = (int32_t*)take(4 * rows);
    c.rseq = (int32_t*)take(4 * rows);
    c.lseq = (int32_t*)take(4 * rows);
    c.lrseq = (int32_t*)take(4 * rows);
    c.sid = (uint32_t*)take(4 * rows);
    c.toff = (uint32_t*)take(4 * rows);
    c.cli = (uint8_t*)take(rows);
    c.rcli = (uint8_t*)take(rows);
    c.flags = (uint8_t*)take(rows);
    c.ng = (uint8_t*)take(rows);
    c.prw = (uint8_t*)take(rows);
    c.ovl = (uint64_t*)take(8 * rows);
    c.pv = (uint16_t*)take(2 * rows * NKEYS);
    c.pk = (uint8_t*)take(rows * NKEYS);
    c.nparent = (int16_t*)take(2 * nodes);
    c.kids = (int16_t*)take(2 * nodes * MAXN);
    c.lorder = (int16_t*)take(2 * nodes);
    c.lpos = (int16_t*)take(2 * nodes);
    c.nchild = (int8_t*)take(nodes);
    c.nlevel = (int8_t*)take(nodes);
    c.nscour = (int8_t*)take(nodes);
    c.hsid = (uint32_t*)take(4 * (int64_t)k.hcap * ndocs);
    c.hseq = (int32_t*)take(4 * (int64_t)k.hcap * ndocs);
    c.mgid = (int32_t*)take(4 * (int64_t)k.mcap * ndocs);
    c.msid = (uint32_t*)take(4 * (int64_t)k.mcap * ndocs);
    c.gq = (int32_t*)take(4 * (int64_t)k.gcap * ndocs);
    c.arena = (uint16_t*)take(2 * 2 * (int64_t)k.acap * ndocs);
    c.s2l = (uint16_t*)take(2 * (int64_t)k.ccap * ndocs);
    c.hdr = (DocHdr*)take(sizeof(DocHdr) * ndocs);
    return off + 256;
}

/* capacity checks shared by every entry point: node ids are int16, heap/log sizes int32 */
inline bool caps_valid(const Caps& k) {
    return k.ncap >= 4 && k.ncap <= 32767 && k.hcap >= 1 && k.acap >= 16 && k.mcap >= 4 && k.gcap >= 1 &&
           k.ccap >= 1 && k.ccap <= 254;
}

} /* namespace mt */
