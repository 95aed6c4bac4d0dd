;; mail-sieve-e.dse -- drop-in replacement for mail-sieve-e.sieve, backed by
;; libdse.so (include/dse.h) through JNA.
;;
;; core.clj calls four functions of the sieve namespace (core.clj:151-152,
;; 163, 192, 196; finish is called by sieve-e itself, sieve.clj:150). This
;; namespace defines them at the same arities and with the same behaviour on
;; the wire and on disk:
;;
;;   spread-work [n num-comps]      sieve.clj:15-34   bounds as Doubles, [[3.0 hi1] [hi1 hi2] ...]
;;   gen-table   [[lower upper]]    sieve.clj:9-13    the chunk (its bounds; no vector is built)
;;   sieve-e     [my-num lead? in-channel chunk out-channel]
;;                                  sieve.clj:118-172 the chunk is sieved on a GPU at once
;;                                  (dse_sieve_odd_range from its bounds); a follower then drains
;;                                  in-channel until machine my-num-1 appoints it; as lead it puts
;;                                  [my-num start prime] for every prime of the chunk (prime a
;;                                  Double in chunk 1) and the appoint [my-num -1 0] on out-channel,
;;                                  so reference machines after it in the ring get what they expect
;;   finish      [raw-chunk my-num] sieve.clj:82-108  user.home/primes{my-num}.txt, byte-exact
;;                                  (dse_write_range_file: chunk 1 as Doubles with the 2/3/5/7 hack)
;;
;; The integration, in core.clj:
;;   (:require ... [mail-sieve-e.sieve :as s] ...)   ->   [mail-sieve-e.dse :as s]   (core.clj:6)
;; and nothing else: the handshake (machine number, [lo hi] bounds, start
;; token, core.clj:154-161,190-194), the relay (core.clj:118-134) and the kill
;; (core.clj:171,199-200) stay the reference's. That covers the reference's own
;; range, N < 2^31 (-main parses N with Integer., core.clj:210). To go past it,
;; two more edits: Long/parseLong for N (core.clj:210) and (mapv long ...) for
;; the follower's bounds (core.clj:191; (int 2.5E10) throws).
;;
;; GPU per machine: the JVM property dse.device if set, else device
;; (my-num - 1) mod (visible devices), so machines 1..8 on one node take GPUs
;; 0..7. jvm/dse_replay.c replays this namespace's libdse calls from C and
;; tests/test_jvm_glue.py runs it on the GPU against the golden files and the
;; reference's lead lines; the image has no JDK, so this file itself is checked
;; statically (every s/ call of core.clj resolves here at its arity).
(ns mail-sieve-e.dse
  (:require [clojure.core.async :refer [>!! <!!]])
  (:import [com.sun.jna Function Memory NativeLibrary Pointer]))

;; ---- libdse.so -------------------------------------------------------------

(def ^:private lib (delay (NativeLibrary/getInstance "dse")))
(defn- f ^Function [^String n] (.getFunction ^NativeLibrary @lib n))

(defn- last-error []
  (.invokeString (f "dse_last_error") (object-array 0) false))

(defn- check [rc where]
  (when-not (zero? (long rc))
    (throw (ex-info (str where ": " (last-error)) {:rc rc :where where}))))

(def ^:private contexts (atom {}))

(defn- context
  "dse_init_device, one context per device for the life of the JVM (the
  reference's process owns its machine for the whole run)."
  ^Pointer [device]
  (locking contexts
    (or (get @contexts device)
        (let [c (.invokePointer (f "dse_init_device") (object-array [(int device)]))]
          (when (nil? c)
            (throw (ex-info (str "dse_init_device: " (last-error)) {:device device})))
          (swap! contexts assoc device c)
          c))))

(defn close!
  "dse_destroy every context this namespace opened."
  []
  (locking contexts
    (doseq [[_ c] @contexts]
      (.invokeVoid (f "dse_destroy") (object-array [c])))
    (reset! contexts {})))

(defn- device-for [my-num]
  (if-let [d (System/getProperty "dse.device")]
    (Integer/parseInt d)
    (let [n (.invokeInt (f "dse_device_count") (object-array 0))]
      (mod (dec (long my-num)) (max 1 n)))))

;; ---- the sieve namespace's interface ---------------------------------------

(defn spread-work
  "sieve.clj:15-34: [[lo hi] ...] for num-comps chunks of floor(floor((n-1)/2)
  / num-comps) odd candidates from 3; the remainder is dropped. Computed in
  exact int64 by dse_spread_work, returned as Doubles like the reference's
  Math/floor arithmetic (the lead writes them on the wire as [5001.0 9999.0])."
  [n num-comps]
  (let [P (int num-comps)
        lo-hi (Memory. (* 16 (max 1 (long P))))
        cs (Memory. 8)]
    (check (.invokeInt (f "dse_spread_work") (object-array [(long n) P lo-hi cs])) "dse_spread_work")
    (vec (for [k (range P)]
           [(double (.getLong lo-hi (* 16 k))) (double (.getLong lo-hi (+ 8 (* 16 k))))]))))

(defn gen-table
  "sieve.clj:9-13: the chunk of odd values [lower, upper). The reference
  materialises them as a transient vector; here the chunk is its bounds plus
  the prime mask sieve-e fills (ceil(cs/64) little-endian longs, bit j = the
  value lower + 2j is prime)."
  [[lower upper]]
  (let [lo (long lower)
        hi (long upper)]
    {:lower lo
     :upper hi
     :doubles? (float? lower)            ; chunk 1 holds Doubles (spread-work's 3.0 head)
     :g-start (quot (- lo 3) 2)
     :nbits (max 0 (quot (- hi lo) 2))  ; (count chunk), sieve.clj:128
     :mask (atom nil)
     :count (atom nil)}))

(defn- sieve-chunk!
  "gen-table + every mark-composites of the chunk (sieve.clj:36-71), on the
  machine's GPU: dse_sieve_odd_range from the chunk's bounds."
  [my-num chunk]
  (when-not @(:mask chunk)
    (let [nb (long (:nbits chunk))
          mask (Memory. (* 8 (max 1 (quot (+ nb 63) 64))))
          cnt (Memory. 8)]
      (check (.invokeInt (f "dse_sieve_odd_range")
                         (object-array [(context (device-for my-num)) (long (:g-start chunk)) nb mask cnt]))
             "dse_sieve_odd_range")
      (reset! (:count chunk) (.getLong cnt 0))
      (reset! (:mask chunk) mask)))
  chunk)

(defn- lead!
  "The lead loop's messages (sieve.clj:131-148): [my-num start prime] for
  every survivor in chunk order -- the primes of the chunk, since every
  smaller prime's multiples are gone by the time this machine leads -- then
  the appoint [my-num -1 0]."
  [my-num chunk out-channel]
  (let [^Memory mask @(:mask chunk)
        nb (long (:nbits chunk))
        lo (long (:lower chunk))
        dbl? (:doubles? chunk)]
    (dotimes [w (quot (+ nb 63) 64)]
      (loop [v (.getLong mask (* 8 w))]
        (when-not (zero? v)
          (let [j (+ (* 64 w) (Long/numberOfTrailingZeros v))]
            (when (< j nb)
              (let [p (+ lo (* 2 j))]
                (>!! out-channel [my-num j (if dbl? (double p) p)])))
            (recur (bit-and v (unchecked-dec v)))))))
    (println "appointing" (inc (long my-num)) "as next machine.")
    (>!! out-channel [my-num -1 0])))

(defn- follow!
  "The follower loop (sieve.clj:154-171) without the marking: the chunk is
  already sieved, so the [mi ps p] lines are read and dropped until machine
  my-num - 1 appoints this one."
  [my-num in-channel]
  (println "Following lead computer...")
  (loop []
    (let [msg (<!! in-channel)]
      (when (nil? msg)
        (throw (ex-info "in-channel closed before this machine was appointed" {:my-num my-num})))
      (let [mi (long (nth msg 0))
            ps (long (nth msg 1))]
        (if (and (= ps -1) (= mi (dec (long my-num))))
          (println "Appointed as new lead.\n")
          (recur))))))

(defn finish
  "sieve.clj:82-108: write user.home/primes{my-num}.txt -- the chunk's primes
  in order, 10 per line, \", \"-separated, LF-terminated; chunk 1 printed as
  Java Doubles with 2.0 3.0 5.0 7.0 first (needs >= 4 candidates)."
  [raw-chunk my-num]
  (println "Writing primes to file...")
  (sieve-chunk! my-num raw-chunk)
  (let [file-name (str (System/getProperty "user.home") "/primes" my-num ".txt")]
    (check (.invokeInt (f "dse_write_range_file")
                       (object-array [file-name (int my-num) (long (:g-start raw-chunk)) (long (:nbits raw-chunk))
                                      @(:mask raw-chunk)]))
           "dse_write_range_file")
    (println "Done!")
    (println "Primes saved in:" file-name "\n")
    (println "")))

(defn sieve-e
  "sieve.clj:118-172 at its arity. The chunk is sieved on the GPU first (a
  follower overlaps that with its wait for the lead); a follower then waits
  for its appoint; the lead's lines go out; finish writes the file."
  [my-num lead? in-channel chunk out-channel]
  (println "Starting Sieve...")
  (sieve-chunk! my-num chunk)
  (when-not lead?
    (follow! my-num in-channel))
  (lead! my-num chunk out-channel)
  (finish chunk my-num))
