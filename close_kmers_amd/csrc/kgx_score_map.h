/* grow_to: a cleared std::unordered_map put in the state the request's map
 * of the reference would be in after holding `most` elements at most
 * (lookup_request.cc keeps one seq_score_ per request and clears it per
 * sequence).  libstdc++ grows the bucket array only when the element count
 * passes what the array holds, and clear() keeps it, so the bucket count --
 * and with it the iteration order of what is inserted next -- follows from
 * the most elements held.  Used to start a part of a request's text on a
 * fresh map; tests/native/score_map_check.cpp checks the claim. */
#pragma once

#include <cstddef>

namespace kgx {

template <typename Map>
void grow_to(Map &m, size_t most)
{
    m.clear();
    for (size_t k = 0; k < most; k++)
        m.emplace((typename Map::key_type)k, typename Map::mapped_type{});
    m.clear();
}

}  // namespace kgx
