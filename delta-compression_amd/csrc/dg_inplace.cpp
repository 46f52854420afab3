// dg_inplace.cpp — in-place delta conversion on the host
// (src/c/inplace.c:272-736, Burns, Long & Stockmeyer, IEEE TKDE 2003).
//
// A graph algorithm over a few thousand COPY commands per delta, so it stays
// on the CPU; it consumes the GPU encoder's output
// (or any standard delta) and emits a delta whose commands can be applied in
// order inside one buffer holding R.
//
// The result must be byte-identical to the reference's, so every ordering
// the reference exposes is reproduced:
//   * CRWI edges i -> j (copy i reads bytes copy j overwrites) are listed per
//     i in destination order: first the write that starts before i's read
//     interval and reaches into it, then the writes starting inside it
//     (inplace.c:387-445);
//   * strongly connected components come from an iterative Tarjan DFS over
//     vertices 0..n-1 with neighbours in list order; an SCC's vertices are
//     in stack-pop order and non-trivial SCCs are visited sources first
//     (:104-222, :470-505);
//   * Kahn's order takes the ready copy with the smallest (length, index)
//     (:517-613); when it stalls the victim is the lowest-index pending copy
//     (constant policy) or the smallest (length, index) copy on the first
//     cycle a resumable DFS finds inside the current SCC (localmin,
//     :227-268, :616-666); the victim becomes an ADD of its R bytes;
//   * output: copies in Kahn order, then the original ADDs in command order,
//     then the converted victims in conversion order (:706-724).
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <vector>

#include "../../include/delta_gpu.h"

namespace {

struct Copy {
	uint64_t src, dst, len;
};
struct Add {
	uint64_t dst, len;
	const uint8_t* data;   // into the input delta or into R
};

constexpr size_t kNone = SIZE_MAX;

uint32_t be32(const uint8_t* p) {
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
void put_be32(std::vector<uint8_t>& o, uint64_t x) {
	o.push_back((uint8_t)(x >> 24));
	o.push_back((uint8_t)(x >> 16));
	o.push_back((uint8_t)(x >> 8));
	o.push_back((uint8_t)x);
}

// Tarjan's SCCs (iterative).  Returns components sinks first, each in the
// order its vertices leave the stack.
void tarjan(const std::vector<std::vector<size_t>>& adj, std::vector<std::vector<size_t>>& comps) {
	const size_t n = adj.size();
	std::vector<size_t> index(n, kNone), low(n, 0), stack;
	std::vector<char> on(n, 0);
	std::vector<std::pair<size_t, size_t>> call;   // (vertex, next neighbour)
	size_t counter = 0;
	for (size_t s = 0; s < n; ++s) {
		if (index[s] != kNone) continue;
		index[s] = low[s] = counter++;
		on[s] = 1;
		stack.push_back(s);
		call.push_back({s, 0});
		while (!call.empty()) {
			const size_t v = call.back().first;
			const size_t ni = call.back().second;
			if (ni < adj[v].size()) {
				const size_t w = adj[v][ni];
				call.back().second++;
				if (index[w] == kNone) {
					index[w] = low[w] = counter++;
					on[w] = 1;
					stack.push_back(w);
					call.push_back({w, 0});
				} else if (on[w] && index[w] < low[v]) {
					low[v] = index[w];
				}
				continue;
			}
			call.pop_back();
			if (!call.empty()) {
				const size_t parent = call.back().first;
				low[parent] = std::min(low[parent], low[v]);
			}
			if (low[v] == index[v]) {
				comps.emplace_back();
				size_t w;
				do {
					w = stack.back();
					stack.pop_back();
					on[w] = 0;
					comps.back().push_back(w);
				} while (w != v);
			}
		}
	}
}

// First cycle reachable inside SCC `sid` among pending vertices, DFS from
// verts[*scan] onwards.  Fully explored vertices stay black (color 2) across
// calls; the grey path is whitened when a cycle is returned.
bool find_cycle(const std::vector<std::vector<size_t>>& adj, const std::vector<size_t>& verts,
                size_t sid, const std::vector<size_t>& scc_id, const std::vector<char>& done,
                std::vector<uint8_t>& color, size_t* scan, std::vector<size_t>& cycle) {
	std::vector<size_t> path;
	std::vector<std::pair<size_t, size_t>> stk;
	for (size_t at = *scan; at < verts.size(); ++at) {
		const size_t start = verts[at];
		if (done[start] || color[start] != 0) continue;
		color[start] = 1;
		path.push_back(start);
		stk.push_back({start, 0});
		while (!stk.empty()) {
			const size_t v = stk.back().first;
			size_t ni = stk.back().second;
			bool pushed = false;
			while (ni < adj[v].size()) {
				const size_t w = adj[v][ni++];
				if (scc_id[w] != sid || done[w]) continue;
				if (color[w] == 1) {   // back edge: the cycle is path[pos..]
					const size_t pos = (size_t)(std::find(path.begin(), path.end(), w) - path.begin());
					cycle.assign(path.begin() + pos, path.end());
					for (size_t x : path) color[x] = 0;
					*scan = at;
					return true;
				}
				if (color[w] == 0) {
					stk.back().second = ni;
					color[w] = 1;
					path.push_back(w);
					stk.push_back({w, 0});
					pushed = true;
					break;
				}
			}
			if (!pushed) {
				stk.pop_back();
				color[v] = 2;
				path.pop_back();
			}
		}
	}
	*scan = verts.size();
	return false;
}

}  // namespace

extern "C" int dg_make_inplace(const uint8_t* r, size_t r_len, const uint8_t* delta,
                               size_t delta_len, int policy, dg_buffer_t* out,
                               dg_inplace_stats_t* stats) {
	if (!out || (delta_len && !delta) || (r_len && !r)) return DG_ERR_INVALID_ARG;
	out->data = nullptr;
	out->len = 0;
	if (stats) memset(stats, 0, sizeof *stats);
	if (delta_len < DG_HEADER_SIZE || memcmp(delta, "DLT\x03", 4) != 0) return DG_ERR_MALFORMED;
	if (delta[4] & 1) {   // already in-place: unchanged (main.c:456-466)
		out->data = (uint8_t*)malloc(delta_len);
		if (!out->data) return DG_ERR_NOMEM;
		memcpy(out->data, delta, delta_len);
		out->len = delta_len;
		if (stats) stats->already_inplace = 1;
		return DG_OK;
	}

	// 1. parse (encoding.c:111-178) and unplace: commands by destination,
	//    stable (apply.c:169-225); a standard delta is already in that order
	struct Parsed {
		int kind;   // 1 COPY, 2 ADD
		uint64_t src, dst, len;
		const uint8_t* data;
	};
	std::vector<Parsed> pc;
	size_t pos = DG_HEADER_SIZE;
	while (pos < delta_len) {
		const uint8_t t = delta[pos++];
		if (t == 0) break;
		if (t == 1) {
			if (pos + 12 > delta_len) return DG_ERR_MALFORMED;
			pc.push_back({1, be32(delta + pos), be32(delta + pos + 4), be32(delta + pos + 8), nullptr});
			pos += 12;
		} else if (t == 2) {
			if (pos + 8 > delta_len) return DG_ERR_MALFORMED;
			const uint64_t d = be32(delta + pos), l = be32(delta + pos + 4);
			pos += 8;
			if (pos + l > delta_len) return DG_ERR_MALFORMED;
			pc.push_back({2, 0, d, l, delta + pos});
			pos += l;
		} else {
			return DG_ERR_MALFORMED;
		}
	}
	std::stable_sort(pc.begin(), pc.end(), [](const Parsed& a, const Parsed& b) { return a.dst < b.dst; });

	// 2. sequential write offsets (inplace.c:296-330)
	std::vector<Copy> copies;
	std::vector<Add> adds;
	uint64_t wpos = 0;
	for (const Parsed& c : pc) {
		if (c.kind == 1) {
			if (c.src + c.len > r_len) return DG_ERR_MALFORMED;   // the victims read R
			copies.push_back({c.src, wpos, c.len});
		} else {
			adds.push_back({wpos, c.len, c.data});
		}
		wpos += c.len;
	}
	const size_t n = copies.size();
	std::vector<size_t> order;   // Kahn order of copies
	if (n) {
		// 3. CRWI digraph: writes sorted by destination, two binary searches
		//    per read interval (inplace.c:346-445)
		std::vector<size_t> by_dst(n);
		for (size_t i = 0; i < n; ++i) by_dst[i] = i;
		std::stable_sort(by_dst.begin(), by_dst.end(),
		                 [&](size_t a, size_t b) { return copies[a].dst < copies[b].dst; });
		std::vector<uint64_t> wstart(n);
		for (size_t k = 0; k < n; ++k) wstart[k] = copies[by_dst[k]].dst;
		std::vector<std::vector<size_t>> adj(n);
		for (size_t i = 0; i < n; ++i) {
			const uint64_t lo_v = copies[i].src, hi_v = copies[i].src + copies[i].len;
			const size_t lo = (size_t)(std::lower_bound(wstart.begin(), wstart.end(), lo_v) - wstart.begin());
			const size_t hi = (size_t)(std::lower_bound(wstart.begin() + lo, wstart.end(), hi_v) - wstart.begin());
			if (lo > 0) {
				const size_t j = by_dst[lo - 1];
				if (j != i && copies[j].dst + copies[j].len > lo_v) adj[i].push_back(j);
			}
			for (size_t k = lo; k < hi; ++k)
				if (by_dst[k] != i) adj[i].push_back(by_dst[k]);
		}

		// 4. SCCs; non-trivial ones sources first (inplace.c:470-505)
		std::vector<std::vector<size_t>> comps;
		tarjan(adj, comps);
		std::vector<size_t> scc_id(n, kNone);
		std::vector<std::vector<size_t>> sccs;
		std::vector<size_t> active;
		for (size_t c = comps.size(); c-- > 0;) {
			if (comps[c].size() <= 1) continue;
			for (size_t v : comps[c]) scc_id[v] = sccs.size();
			active.push_back(comps[c].size());
			sccs.push_back(std::move(comps[c]));
		}

		// 5. Kahn with (length, index) priority and cycle breaking
		std::vector<size_t> indeg(n, 0);
		for (size_t i = 0; i < n; ++i)
			for (size_t w : adj[i]) indeg[w]++;
		using Key = std::pair<uint64_t, size_t>;
		std::priority_queue<Key, std::vector<Key>, std::greater<Key>> ready;
		for (size_t i = 0; i < n; ++i)
			if (indeg[i] == 0) ready.push({copies[i].len, i});
		std::vector<char> done(n, 0);
		std::vector<uint8_t> color(n, 0);
		size_t scc_ptr = 0, scan = 0, processed = 0;
		std::vector<size_t> cycle;
		auto retire = [&](size_t v) {
			done[v] = 1;
			++processed;
			if (scc_id[v] != kNone) active[scc_id[v]]--;
			for (size_t w : adj[v])
				if (!done[w] && --indeg[w] == 0) ready.push({copies[w].len, w});
		};
		order.reserve(n);
		while (processed < n) {
			while (!ready.empty()) {
				const size_t v = ready.top().second;
				ready.pop();
				if (done[v]) continue;
				order.push_back(v);
				retire(v);
			}
			if (processed >= n) break;
			size_t victim = kNone;
			if (policy == DG_POLICY_CONSTANT) {
				for (size_t i = 0; i < n && victim == kNone; ++i)
					if (!done[i]) victim = i;
			} else {
				while (victim == kNone) {
					while (scc_ptr < sccs.size() && active[scc_ptr] == 0) {
						++scc_ptr;
						scan = 0;
					}
					if (scc_ptr >= sccs.size()) {   // safety fallback (inplace.c:634-640)
						for (size_t i = 0; i < n && victim == kNone; ++i)
							if (!done[i]) victim = i;
						break;
					}
					if (find_cycle(adj, sccs[scc_ptr], scc_ptr, scc_id, done, color, &scan, cycle)) {
						victim = cycle[0];
						for (size_t v : cycle)
							if (copies[v].len < copies[victim].len ||
							    (copies[v].len == copies[victim].len && v < victim))
								victim = v;
					} else {
						++scc_ptr;
						scan = 0;
					}
				}
			}
			adds.push_back({copies[victim].dst, copies[victim].len, r + copies[victim].src});
			retire(victim);
		}
	}

	// 6. encode (encoding.c:39-90): copies in order, then the ADDs
	std::vector<uint8_t> o;
	uint64_t add_bytes = 0;
	for (const Add& a : adds) add_bytes += a.len;
	o.reserve(DG_HEADER_SIZE + 13 * order.size() + 9 * adds.size() + add_bytes + 1);
	o.insert(o.end(), delta, delta + 4);
	o.push_back(1);                                   // DELTA_FLAG_INPLACE
	o.insert(o.end(), delta + 5, delta + DG_HEADER_SIZE);   // version size + both CRCs
	uint64_t copy_bytes = 0;
	for (size_t v : order) {
		o.push_back(1);
		put_be32(o, copies[v].src);
		put_be32(o, copies[v].dst);
		put_be32(o, copies[v].len);
		copy_bytes += copies[v].len;
	}
	for (const Add& a : adds) {
		o.push_back(2);
		put_be32(o, a.dst);
		put_be32(o, a.len);
		o.insert(o.end(), a.data, a.data + a.len);
	}
	o.push_back(0);
	out->data = (uint8_t*)malloc(o.size());
	if (!out->data) return DG_ERR_NOMEM;
	memcpy(out->data, o.data(), o.size());
	out->len = o.size();
	if (stats) {
		stats->num_copies = order.size();
		stats->num_adds = adds.size();
		stats->copy_bytes = copy_bytes;
		stats->add_bytes = add_bytes;
	}
	return DG_OK;
}
