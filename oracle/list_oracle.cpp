// list_oracle.cpp — CPU restatement of the window-contents (ListState) paths: WindowedStream.apply/process
// (WindowOperator + ListStateDescriptor + InternalIterableWindowFunction) and the EvictingWindowOperator.
// TEST INFRASTRUCTURE ONLY; see list_oracle.h for the reference files restated.  Paths below are relative to
// /root/reference/flink-streaming-java/src/main/java/org/apache/flink/streaming/.
#include "list_oracle.h"

#include "window_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <queue>
#include <set>
#include <vector>

namespace {

const int64_t LMAX = INT64_MAX;
const int64_t LMIN = INT64_MIN;
inline int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
inline double bitsd(int64_t b) {
  double d;
  memcpy(&d, &b, 8);
  return d;
}
inline int64_t dbits_raw(double d) {
  int64_t b;
  memcpy(&b, &d, 8);
  return b;
}
inline int64_t dbits(double d) { return std::isnan(d) ? 0x7ff8000000000000LL : dbits_raw(d); }
// Double.compare (Float.compare of floats widened to double orders the same way)
inline int jcmp(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  const int64_t x = dbits(a), y = dbits(b);
  return x == y ? 0 : (x < y ? -1 : 1);
}
// TimeWindow.java:254-256
inline int64_t window_start(int64_t ts, int64_t offset, int64_t size) {
  const int64_t t = jadd(jsub(ts, offset), size);
  return jsub(ts, t % size);
}

struct OpErr {
  int code;
};

struct W {
  int64_t start, end;
  int64_t max_ts() const { return end == LMAX && start == LMIN ? LMAX : jsub(end, 1); }  // GlobalWindow: MAX
  bool operator<(const W& o) const { return start != o.start ? start < o.start : end < o.end; }
  bool operator==(const W& o) const { return start == o.start && end == o.end; }
};
struct KW {
  int64_t key;
  W w;
  bool operator<(const KW& o) const { return key != o.key ? key < o.key : w < o.w; }
};
struct Timer {
  int64_t ts;
  KW kw;
  bool operator<(const Timer& o) const { return ts != o.ts ? ts < o.ts : kw < o.kw; }
  bool operator>(const Timer& o) const { return o < *this; }
};
struct Elem {
  int64_t ts, val, ord;
};

// ---------------------------------------------------------------- merging windows (EventTimeSessionWindows)
// TimeWindow.hashCode = MathUtils.longToIntWithBitMixing(start + end) (TimeWindow.java:102-104, MathUtils.java:177-182)
inline int32_t tw_hash(const W& w) {
  uint64_t in = (uint64_t)jadd(w.start, w.end);
  in = (in ^ (in >> 30)) * 0xbf58476d1ce4e5b9ULL;
  in = (in ^ (in >> 27)) * 0x94d049bb133111ebULL;
  in = in ^ (in >> 31);
  return (int32_t)in;
}
// iteration order of a java.util.HashSet<TimeWindow> that had `ins` added in this order (TimeWindow.mergeWindows'
// merge sets, TimeWindow.java:213-233): HashMap buckets (h ^ h >>> 16) & (capacity - 1), capacity 16 doubled past 3/4
// load, a bucket in insertion order (a resize splits buckets keeping it; the small sets of a session merge never
// treeify)
std::vector<W> hashset_order(const std::vector<W>& ins) {
  size_t cap = 16;
  while (ins.size() > cap * 3 / 4) cap *= 2;
  std::vector<std::pair<uint32_t, size_t>> k(ins.size());
  for (size_t i = 0; i < ins.size(); i++) {
    const uint32_t h = (uint32_t)tw_hash(ins[i]);
    k[i] = {(h ^ (h >> 16)) & (uint32_t)(cap - 1), i};
  }
  std::sort(k.begin(), k.end());
  std::vector<W> out;
  for (const auto& x : k) out.push_back(ins[x.second]);
  return out;
}

struct ListOracle {
  explicit ListOracle(const oracle_list_cfg& c) : cfg(c) {}
  oracle_list_cfg cfg;
  int64_t wm = LMIN, epoch = 0, ordinal = -1, late_dropped = 0;
  std::map<KW, std::vector<Elem>> lists;  // "window-contents"
  std::map<KW, int64_t> counts;           // CountTrigger's ReducingState "count"
  std::set<Timer> timer_set;
  std::priority_queue<Timer, std::vector<Timer>, std::greater<Timer>> timer_q;
  std::vector<oracle_list_row> rows;
  std::vector<oracle_list_elem> elems;
  std::vector<int64_t> side_key, side_ts, side_val, side_epoch;

  bool event_time() const { return cfg.assigner != OR_GLOBAL; }  // GlobalWindows.isEventTime() == false
  bool merging() const { return cfg.assigner == OR_SESSION; }     // (cfg.size = the session gap)
  std::map<int64_t, std::map<W, W>> msets;                       // MergingWindowSet per key: window -> state window
  bool is_float() const { return cfg.value_type == OR_VAL_F64 || cfg.value_type == OR_VAL_F32; }

  // WindowOperator.java:576-651
  int64_t cleanup_time(const W& w) const {
    if (!event_time()) return w.max_ts();
    const int64_t c = jadd(w.max_ts(), cfg.lateness);
    return c >= w.max_ts() ? c : LMAX;
  }
  bool is_window_late(const W& w) const { return event_time() && cleanup_time(w) <= wm; }
  bool is_element_late(int64_t ts) const { return event_time() && jadd(ts, cfg.lateness) <= wm; }
  void register_timer(int64_t ts, const KW& kw) {
    const Timer t{ts, kw};
    if (timer_set.insert(t).second) timer_q.push(t);
  }
  void register_cleanup_timer(const KW& kw) {
    const int64_t c = cleanup_time(kw.w);
    if (c == LMAX) return;
    register_timer(c, kw);
  }
  void delete_timer(int64_t ts, const KW& kw) { timer_set.erase(Timer{ts, kw}); }

  // MergingWindowSet.addWindow (MergingWindowSet.java:150-225) with TimeWindow.mergeWindows (TimeWindow.java:201-244)
  // and EvictingWindowOperator's merge function (:118-148): the windows in flight are pairwise non-touching, so the
  // one merge set (if any) holds the new window; its state window is the first merged window's in HashSet order,
  // and the others' lists are appended to it in that order (HeapListState.mergeState = addAll,
  // AbstractHeapMergingState.mergeNamespaces :67-93).
  W add_window(int64_t key, std::map<W, W>& mapping, const W& nw) {
    std::vector<W> ws;
    for (const auto& kv : mapping) ws.push_back(kv.first);
    ws.push_back(nw);
    std::stable_sort(ws.begin(), ws.end(), [](const W& a, const W& b) { return a.start < b.start; });
    std::vector<std::pair<W, std::vector<W>>> merged;  // (cover, members in insertion order)
    for (const W& c : ws) {
      if (!merged.empty() && merged.back().first.start <= c.end && merged.back().first.end >= c.start) {  // intersects
        W& cv = merged.back().first;
        cv = W{std::min(cv.start, c.start), std::max(cv.end, c.end)};
        merged.back().second.push_back(c);
      } else {
        merged.push_back({c, {c}});
      }
    }
    W result = nw;
    bool merged_new = false, any = false;
    for (auto& m : merged) {
      if (m.second.size() < 2) continue;
      any = true;
      const W mr = m.first;
      std::vector<W> mws = hashset_order(m.second);
      const auto it_new = std::find(mws.begin(), mws.end(), nw);
      if (it_new != mws.end()) {
        mws.erase(it_new);
        merged_new = true;
        result = mr;
      }
      const W target = mapping.at(mws.front());
      std::vector<W> sources;
      for (const W& w : mws) {
        auto it = mapping.find(w);
        if (it != mapping.end()) {
          sources.push_back(it->second);
          mapping.erase(it);
        }
      }
      mapping[mr] = target;
      const auto it_t = std::find(sources.begin(), sources.end(), target);
      if (it_t != sources.end()) sources.erase(it_t);
      if (!(std::find(mws.begin(), mws.end(), mr) != mws.end() && mws.size() == 1)) {
        if (jadd(mr.max_ts(), cfg.lateness) <= wm) throw OpErr{OR_ERR_MERGE_LATE};
        register_timer(mr.max_ts(), KW{key, mr});  // EventTimeTrigger.onMerge
        for (const W& w : mws) {
          delete_timer(w.max_ts(), KW{key, w});  // triggerContext.clear() -> EventTimeTrigger.clear
          const int64_t c = cleanup_time(w);
          if (c != LMAX) delete_timer(c, KW{key, w});  // deleteCleanupTimer
        }
        for (const W& src : sources) {  // mergeNamespaces(target, sources)
          auto it = lists.find(KW{key, src});
          if (it == lists.end()) continue;
          std::vector<Elem> moved = std::move(it->second);
          lists.erase(it);
          std::vector<Elem>& t = lists[KW{key, target}];
          t.insert(t.end(), moved.begin(), moved.end());
        }
      }
    }
    if (!any || (result == nw && !merged_new)) mapping[result] = result;
    return result;
  }

  void assign(int64_t ts, std::vector<W>& out) const {
    out.clear();
    if (cfg.assigner == OR_GLOBAL) {  // GlobalWindows.assignWindows: the one GlobalWindow
      out.push_back(W{LMIN, LMAX});
      return;
    }
    if (ts == LMIN) throw OpErr{OR_ERR_NO_TIMESTAMP};  // TumblingEventTimeWindows.java:69-71
    if (cfg.assigner == OR_TUMBLING) {
      const int64_t s = window_start(ts, cfg.offset, cfg.size);
      out.push_back(W{s, jadd(s, cfg.size)});
      return;
    }
    const int64_t last = window_start(ts, cfg.offset, cfg.slide);  // SlidingEventTimeWindows.java:67-81
    for (int64_t s = last; s > jsub(ts, cfg.size); s = jsub(s, cfg.slide)) out.push_back(W{s, jadd(s, cfg.size)});
  }

  // DeltaEvictor's built-in DeltaFunction: last.field - e.field in the field's Java arithmetic
  double delta(int64_t e, int64_t last) const {
    switch (cfg.value_type) {
      case OR_VAL_I64: return (double)jsub(last, e);
      case OR_VAL_F64: return bitsd(last) - bitsd(e);
      case OR_VAL_F32: return (double)((float)bitsd(last) - (float)bitsd(e));
      default: return (double)(int32_t)(uint32_t)((uint32_t)(int32_t)last - (uint32_t)(int32_t)e);
    }
  }
  // CountEvictor.evict (:63-78), TimeEvictor.evict (:75-103), DeltaEvictor.evict (:71-80)
  void evict(std::vector<Elem>& l) const {
    if (cfg.evictor == OR_EVICT_COUNT) {
      if ((int64_t)l.size() <= cfg.evict_count) return;
      l.erase(l.begin(), l.begin() + ((int64_t)l.size() - cfg.evict_count));
    } else if (cfg.evictor == OR_EVICT_TIME) {
      if (l.empty() || l.front().ts == LMIN) return;  // hasTimestamp of the first element
      int64_t cur = LMIN;
      for (const Elem& e : l) cur = std::max(cur, e.ts);
      const int64_t cutoff = jsub(cur, cfg.evict_count);
      std::vector<Elem> keep;
      for (const Elem& e : l)
        if (!(e.ts <= cutoff)) keep.push_back(e);
      l.swap(keep);
    } else if (cfg.evictor == OR_EVICT_DELTA) {
      if (l.empty()) return;
      const int64_t last = l.back().val;
      std::vector<Elem> keep;
      for (const Elem& e : l)
        if (!(delta(e.val, last) >= cfg.delta_threshold)) keep.push_back(e);
      l.swap(keep);
    }
  }

  // EvictingWindowOperator.emitWindowContents (:334-366): evictBefore, the function over the remaining
  // elements (recorded as a row and its contents), evictAfter, and the list re-stored (empty: cleared).
  // kw: the window the row reports; lkw: the list's namespace (the state window of a merging window)
  void emit_contents(const KW& kw) { emit_contents(kw, kw); }
  void emit_contents(const KW& kw, const KW& lkw) {
    std::vector<Elem>& l = lists[lkw];
    if (!cfg.evict_after) evict(l);
    oracle_list_row r{};
    r.key = kw.key;
    r.start = kw.w.start;
    r.end = kw.w.end;
    r.count = (int64_t)l.size();
    r.first = l.empty() ? -1 : l.front().ord;
    r.elem_off = (int64_t)elems.size();
    r.epoch = epoch;
    double ds = 0.0, dmn = 0.0, dmx = 0.0;
    int64_t is = 0, imn = 0, imx = 0;
    bool first = true;
    for (const Elem& e : l) {
      elems.push_back(oracle_list_elem{e.ts, e.val, e.ord});
      if (is_float()) {
        const double d = bitsd(e.val);
        ds = first ? d : cfg.value_type == OR_VAL_F32 ? (double)((float)ds + (float)d) : ds + d;
        if (first || jcmp(d, dmn) < 0) dmn = d;
        if (first || jcmp(d, dmx) > 0) dmx = d;
      } else {
        is = first ? e.val : jadd(is, e.val);
        if (first || e.val < imn) imn = e.val;
        if (first || e.val > imx) imx = e.val;
      }
      first = false;
    }
    if (is_float()) {
      r.sum = dbits_raw(ds);
      r.min = l.empty() ? 0 : dbits(dmn);
      r.max = l.empty() ? 0 : dbits(dmx);
    } else {
      r.sum = cfg.value_type == OR_VAL_I32 ? (int64_t)(int32_t)is : cfg.value_type == OR_VAL_I16 ? (int64_t)(int16_t)is
            : cfg.value_type == OR_VAL_I8 ? (int64_t)(int8_t)is : is;
      r.min = imn;
      r.max = imx;
    }
    rows.push_back(r);
    if (cfg.evict_after) evict(l);
    if (l.empty()) lists.erase(lkw);  // windowState.clear() and nothing re-added
  }

  // EvictingWindowOperator.processElement, merging branch (:110-170)
  void process_merging(int64_t key, int64_t ts, int64_t val) {
    std::map<W, W>& mapping = msets[key];
    const W nw{ts, jadd(ts, cfg.size)};  // EventTimeSessionWindows.assignWindows
    const W actual = add_window(key, mapping, nw);
    if (is_window_late(actual)) {
      mapping.erase(actual);  // MergingWindowSet.retireWindow
    } else {
      const KW lkw{key, mapping.at(actual)}, akw{key, actual};
      lists[lkw].push_back(Elem{ts, val, ordinal});
      bool fire = false;
      if (actual.max_ts() <= wm)  // EventTimeTrigger.onElement
        fire = true;
      else
        register_timer(actual.max_ts(), akw);
      if (fire) emit_contents(akw, lkw);
      if (fire && cfg.purging) lists.erase(lkw);
      register_cleanup_timer(akw);
      if (mapping.empty()) msets.erase(key);
      return;
    }
    if (mapping.empty()) msets.erase(key);
    if (is_element_late(ts)) {
      if (cfg.side_output) {
        side_key.push_back(key);
        side_ts.push_back(ts);
        side_val.push_back(val);
        side_epoch.push_back(epoch);
      } else {
        late_dropped++;
      }
    }
  }

  // EvictingWindowOperator.processElement, non-merging branch (:186-222) / WindowOperator.java:379-407
  std::vector<W> wbuf;
  void process_element(int64_t key, int64_t ts, int64_t val) {
    ordinal++;
    if (merging()) {
      process_merging(key, ts, val);
      return;
    }
    assign(ts, wbuf);
    bool skipped = true;
    for (const W& w : wbuf) {
      if (is_window_late(w)) continue;
      skipped = false;
      const KW kw{key, w};
      lists[kw].push_back(Elem{ts, val, ordinal});
      bool fire = false;
      if (cfg.trigger == OR_TRIG_COUNT) {  // CountTrigger.onElement (:47-55)
        int64_t& c = counts[kw];
        if (++c >= cfg.trigger_count) {
          counts.erase(kw);
          fire = true;
        }
      } else {  // EventTimeTrigger.onElement (:37-45)
        if (w.max_ts() <= wm)
          fire = true;
        else
          register_timer(w.max_ts(), kw);
      }
      if (fire) emit_contents(kw);
      if (fire && cfg.purging) lists.erase(kw);  // PurgingTrigger: FIRE_AND_PURGE
      register_cleanup_timer(kw);
    }
    if (skipped && is_element_late(ts)) {
      if (cfg.side_output) {
        side_key.push_back(key);
        side_ts.push_back(ts);
        side_val.push_back(val);
        side_epoch.push_back(epoch);
      } else {
        late_dropped++;
      }
    }
  }

  // EvictingWindowOperator.onEventTime (:241-286)
  void on_event_time(const Timer& t) {
    const KW& kw = t.kw;
    if (merging()) {  // EvictingWindowOperator.onEventTime (:241-286) with the window's state window
      auto ms = msets.find(kw.key);
      if (ms == msets.end()) return;
      auto it = ms->second.find(kw.w);
      if (it == ms->second.end()) return;  // (a timer of a window no longer in flight)
      const KW lkw{kw.key, it->second};
      if (lists.count(lkw)) {
        const bool fire = t.ts == kw.w.max_ts();
        if (fire) emit_contents(kw, lkw);
        if (fire && cfg.purging) lists.erase(lkw);
      }
      if (t.ts == cleanup_time(kw.w)) {  // clearAllState: contents, trigger timer, retireWindow
        lists.erase(lkw);
        timer_set.erase(Timer{kw.w.max_ts(), kw});
        ms->second.erase(kw.w);
        if (ms->second.empty()) msets.erase(ms);
      }
      return;
    }
    if (lists.count(kw)) {
      const bool fire = cfg.trigger == OR_TRIG_EVENT_TIME && t.ts == kw.w.max_ts();  // EventTimeTrigger.onEventTime
      if (fire) emit_contents(kw);
      if (fire && cfg.purging) lists.erase(kw);
    }
    if (event_time() && t.ts == cleanup_time(kw.w)) {  // clearAllState: contents, trigger state and timer
      lists.erase(kw);
      counts.erase(kw);
      if (cfg.trigger == OR_TRIG_EVENT_TIME) timer_set.erase(Timer{kw.w.max_ts(), kw});
    }
  }

  void process_watermark(int64_t w) {
    wm = w;
    while (!timer_q.empty() && timer_q.top().ts <= w) {
      const Timer t = timer_q.top();
      timer_q.pop();
      auto it = timer_set.find(t);
      if (it == timer_set.end()) continue;  // deleted
      timer_set.erase(it);
      on_event_time(t);
    }
    epoch++;
  }
};

}  // namespace

extern "C" {

void* oracle_list_create(const oracle_list_cfg* cfg) {
  if (cfg->assigner != OR_GLOBAL && cfg->assigner != OR_TUMBLING && cfg->assigner != OR_SLIDING &&
      cfg->assigner != OR_SESSION)
    return nullptr;
  if (cfg->assigner == OR_SESSION && cfg->trigger != OR_TRIG_EVENT_TIME) return nullptr;  // (EventTimeTrigger only)
  if (cfg->assigner != OR_GLOBAL && cfg->size <= 0) return nullptr;
  if (cfg->assigner == OR_SLIDING && cfg->slide <= 0) return nullptr;
  if (cfg->trigger == OR_TRIG_COUNT && cfg->trigger_count <= 0) return nullptr;
  return new ListOracle(*cfg);
}
void oracle_list_destroy(void* op) { delete static_cast<ListOracle*>(op); }
int oracle_list_process(void* p, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n) {
  auto* o = static_cast<ListOracle*>(p);
  try {
    for (int64_t i = 0; i < n; i++) o->process_element(key[i], ts[i], val[i]);
  } catch (const OpErr& e) {
    return e.code;
  }
  return OR_OK;
}
int oracle_list_watermark(void* p, int64_t wm) {
  static_cast<ListOracle*>(p)->process_watermark(wm);
  return OR_OK;
}
int64_t oracle_list_num_rows(void* p) { return (int64_t)static_cast<ListOracle*>(p)->rows.size(); }
int64_t oracle_list_num_elems(void* p) { return (int64_t)static_cast<ListOracle*>(p)->elems.size(); }
void oracle_list_get_rows(void* p, oracle_list_row* out) {
  auto* o = static_cast<ListOracle*>(p);
  std::copy(o->rows.begin(), o->rows.end(), out);
}
void oracle_list_get_elems(void* p, oracle_list_elem* out) {
  auto* o = static_cast<ListOracle*>(p);
  std::copy(o->elems.begin(), o->elems.end(), out);
}
int64_t oracle_list_num_side_rows(void* p) { return (int64_t)static_cast<ListOracle*>(p)->side_key.size(); }
void oracle_list_get_side_rows(void* p, int64_t* key, int64_t* ts, int64_t* val, int64_t* epoch) {
  auto* o = static_cast<ListOracle*>(p);
  std::copy(o->side_key.begin(), o->side_key.end(), key);
  std::copy(o->side_ts.begin(), o->side_ts.end(), ts);
  std::copy(o->side_val.begin(), o->side_val.end(), val);
  std::copy(o->side_epoch.begin(), o->side_epoch.end(), epoch);
}
int64_t oracle_list_late_dropped(void* p) { return static_cast<ListOracle*>(p)->late_dropped; }
int64_t oracle_list_num_state_entries(void* p) { return (int64_t)static_cast<ListOracle*>(p)->lists.size(); }
int64_t oracle_list_num_timers(void* p) { return (int64_t)static_cast<ListOracle*>(p)->timer_set.size(); }

}  // extern "C"
