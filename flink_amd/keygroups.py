"""Host mirror of KeyGroupRangeAssignment / KeyGroupRange / MathUtils.murmurHash for scalar,
control-plane use (deciding which KeyGroupRange a subtask owns, routing a single key).  The
per-record versions run on the GPU (fw_key_groups_device / fw_route_device).

Reference: flink-runtime/src/main/java/org/apache/flink/runtime/state/KeyGroupRangeAssignment.java:47-135,
flink-runtime/src/main/java/org/apache/flink/runtime/state/KeyGroupRange.java:30-189,
flink-core/src/main/java/org/apache/flink/util/MathUtils.java:134-198.
"""
DEFAULT_LOWER_BOUND_MAX_PARALLELISM = 1 << 7  # KeyGroupRangeAssignment.java:30
UPPER_BOUND_MAX_PARALLELISM = 1 << 15         # KeyGroupRangeAssignment.java:33

_M32 = 0xFFFFFFFF


def _i32(x):
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def _rotl(x, r):
    x &= _M32
    return ((x << r) | (x >> (32 - r))) & _M32


def bit_mix(v):
    """MathUtils.bitMix (MathUtils.java:191-198)."""
    x = v & _M32
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & _M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & _M32
    x ^= x >> 16
    return _i32(x)


def murmur_hash(code):
    """MathUtils.murmurHash (MathUtils.java:134-154): non-negative 32-bit hash."""
    c = (code * 0xCC9E2D51) & _M32
    c = _rotl(c, 15)
    c = (c * 0x1B873593) & _M32
    c = _rotl(c, 13)
    c = (c * 5 + 0xE6546B64) & _M32
    c ^= 4
    r = bit_mix(c)
    if r >= 0:
        return r
    return -r if r != -(1 << 31) else 0


def long_hash_code(v):
    """Long.hashCode: (int)(value ^ (value >>> 32))."""
    v &= (1 << 64) - 1
    return _i32(v ^ (v >> 32))


def string_hash_code(s):
    """String.hashCode over UTF-16 code units: s[0]*31^(n-1) + ... + s[n-1]."""
    b = s.encode("utf-16-be")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + ((b[i] << 8) | b[i + 1])) & _M32
    return _i32(h)


def string_key_id(s):
    """The key column's 64-bit identity of a String key decoded from the wire (fw_wire_decode_keyed_device):
    FNV-1a 64 over the UTF-16 chars, then fmix64 of it ^ the char count, as a signed long."""
    b = s.encode("utf-16-le")
    f = 0xcbf29ce484222325
    for i in range(0, len(b), 2):
        f = ((f ^ (b[i] | (b[i + 1] << 8))) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    x = f ^ (len(b) // 2)
    x ^= x >> 33
    x = (x * 0xff51afd7ed558ccd) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 33
    x = (x * 0xc4ceb9fe1a85ec53) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 33
    return x - (1 << 64) if x >= (1 << 63) else x


def compute_key_group_for_key_hash(key_hash, max_parallelism):
    """KeyGroupRangeAssignment.computeKeyGroupForKeyHash (:69-71)."""
    return murmur_hash(key_hash) % max_parallelism


def assign_to_key_group(key_hash, max_parallelism):
    """KeyGroupRangeAssignment.assignToKeyGroup(key, maxPar) given key.hashCode() (:58-60)."""
    return compute_key_group_for_key_hash(key_hash, max_parallelism)


def check_parallelism_preconditions(parallelism):
    if not (0 < parallelism <= UPPER_BOUND_MAX_PARALLELISM):
        raise ValueError(f"Operator parallelism not within bounds: {parallelism}")


def compute_key_group_range_for_operator_index(max_parallelism, parallelism, operator_index):
    """KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex (:85-99)."""
    check_parallelism_preconditions(parallelism)
    check_parallelism_preconditions(max_parallelism)
    if max_parallelism < parallelism:
        raise ValueError("Maximum parallelism must not be smaller than parallelism.")
    start = (operator_index * max_parallelism + parallelism - 1) // parallelism
    end = ((operator_index + 1) * max_parallelism - 1) // parallelism
    return KeyGroupRange(start, end)


def compute_operator_index_for_key_group(max_parallelism, parallelism, key_group_id):
    """KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup (:115-117)."""
    return key_group_id * parallelism // max_parallelism


def assign_key_to_parallel_operator(key_hash, max_parallelism, parallelism):
    """KeyGroupRangeAssignment.assignKeyToParallelOperator (:47-49)."""
    return compute_operator_index_for_key_group(max_parallelism, parallelism,
                                                assign_to_key_group(key_hash, max_parallelism))


def round_up_to_power_of_two(x):
    """MathUtils.roundUpToPowerOfTwo."""
    x -= 1
    for s in (1, 2, 4, 8, 16):
        x |= x >> s
    return x + 1


def compute_default_max_parallelism(operator_parallelism):
    """KeyGroupRangeAssignment.computeDefaultMaxParallelism (:126-135)."""
    check_parallelism_preconditions(operator_parallelism)
    return min(max(round_up_to_power_of_two(operator_parallelism + operator_parallelism // 2),
                   DEFAULT_LOWER_BOUND_MAX_PARALLELISM), UPPER_BOUND_MAX_PARALLELISM)


class KeyGroupRange:
    """Inclusive range of key groups (KeyGroupRange.java:30-189); empty when end < start."""

    def __init__(self, start, end):
        if start < 0 or (end >= 0 and end < start - 1):
            raise ValueError("Invalid key group range")
        self.start_key_group = start
        self.end_key_group = end

    @staticmethod
    def of(start, end):
        return KeyGroupRange(start, end)

    def contains(self, key_group):
        return self.start_key_group <= key_group <= self.end_key_group

    def get_number_of_key_groups(self):
        return max(0, self.end_key_group - self.start_key_group + 1)

    def get_intersection(self, other):
        start = max(self.start_key_group, other.start_key_group)
        end = min(self.end_key_group, other.end_key_group)
        return KeyGroupRange(start, end) if start <= end else KeyGroupRange(0, -1)

    def __iter__(self):
        return iter(range(self.start_key_group, self.end_key_group + 1))

    def __eq__(self, other):
        return isinstance(other, KeyGroupRange) and (self.start_key_group, self.end_key_group) == (
            other.start_key_group, other.end_key_group)

    def __repr__(self):
        return f"KeyGroupRange{{startKeyGroup={self.start_key_group}, endKeyGroup={self.end_key_group}}}"
