;; mail-sieve-e.dse -- the reference's hot path behind libdse.so (include/dse.h).
;;
;; Drop-in for the sieve calls of core.clj: lead-start (core.clj:136-179) and
;; client-start (core.clj:181-205) call s/spread-work, s/gen-table and
;; s/sieve-e (core.clj:151-152,163,192,196), and sieve-e ends in finish
;; (sieve.clj:150). With this namespace they call the C ABI through JNA
;; instead; the per-prime [mi ps p] relay (sieve.clj:139, core.clj:118-134)
;; is not needed, since every machine sieves its whole chunk on its GPU.
;;
;; The same call sequence, from C, is jvm/dse_replay.c; tests/test_jvm_glue.py
;; runs it on the GPU and checks the files against the golden hashes.
(ns mail-sieve-e.dse
  (:import [com.sun.jna Function Memory NativeLibrary Pointer]))

(def ^:private lib (delay (NativeLibrary/getInstance "dse")))
(defn- f ^Function [^String n] (.getFunction ^NativeLibrary @lib n))

(defn- last-error []
  (.invokeString (f "dse_last_error") (object-array 0) false))

(defn- check [rc where]
  (when-not (zero? rc)
    (throw (ex-info (str where ": " (last-error)) {:rc rc :where where}))))

(defn init
  "dse_init: one context over num-gpus devices (replaces the socket server and
  the client wait, core.clj:76-116)."
  ^Pointer [num-gpus]
  (let [^Pointer ctx (.invokePointer (f "dse_init") (object-array [(int num-gpus)]))]
    (when (nil? ctx) (throw (ex-info (str "dse_init: " (last-error)) {})))
    ctx))

(defn destroy [^Pointer ctx]
  (.invokeVoid (f "dse_destroy") (object-array [ctx])))

(defn spread-work
  "sieve.clj:15-34 in exact longs: [[lo hi] ...] and the chunk size."
  [n num-comps]
  (let [lo-hi (Memory. (* 16 (long num-comps)))
        cs (Memory. 8)]
    (check (.invokeInt (f "dse_spread_work") (object-array [(long n) (int num-comps) lo-hi cs]))
           "dse_spread_work")
    {:chunks (vec (for [k (range num-comps)]
                    [(.getLong lo-hi (* 16 k)) (.getLong lo-hi (+ 8 (* 16 k)))]))
     :cs (.getLong cs 0)}))

(defn sieve-chunk!
  "gen-table + sieve-e for machine my-num (sieve.clj:9-13,118-172): the chunk's
  odd-only prime mask (ceil(cs/64) little-endian longs) and its prime count."
  [^Pointer ctx n num-comps my-num cs]
  (let [mask (Memory. (* 8 (quot (+ (long cs) 63) 64)))
        cnt (Memory. 8)]
    (check (.invokeInt (f "dse_sieve_chunk")
                       (object-array [ctx (long n) (int num-comps) (int my-num) mask cnt]))
           "dse_sieve_chunk")
    {:mask mask :count (.getLong cnt 0)}))

(defn finish!
  "sieve.clj:82-108: write user.home/primes{my-num}.txt byte-exactly (chunk 1
  as Doubles with the 2/3/5/7 hack)."
  ([my-num n num-comps mask]
   (finish! (str (System/getProperty "user.home") "/primes" my-num ".txt") my-num n num-comps mask))
  ([^String path my-num n num-comps mask]
   (check (.invokeInt (f "dse_write_primes_file")
                      (object-array [path (int my-num) (long n) (int num-comps) mask]))
          "dse_write_primes_file")
   path))

(defn run-machine!
  "What lead-start (my-num 1, core.clj:151-152,163) and client-start (its
  machine number, core.clj:192,196) do with the sieve, in the order the C
  replay makes the calls: dse_init -> dse_spread_work -> dse_sieve_chunk ->
  dse_write_primes_file -> dse_destroy. Returns the prime count of the chunk."
  ([my-num num-primes num-expected]
   (run-machine! my-num num-primes num-expected nil))
  ([my-num num-primes num-expected out-dir]
   (let [ctx (init 1)]
     (try
       (let [{:keys [cs]} (spread-work num-primes num-expected)
             {:keys [mask count]} (sieve-chunk! ctx num-primes num-expected my-num cs)]
         (if out-dir
           (finish! (str out-dir "/primes" my-num ".txt") my-num num-primes num-expected mask)
           (finish! my-num num-primes num-expected mask))
         count)
       (finally (destroy ctx))))))

;; In core.clj (the maintainer's edit):
;;   lead-start:   replace (s/spread-work ...) / (s/gen-table ...) / (s/sieve-e 1 true ...)
;;                 (core.clj:151-152,163) by (dse/run-machine! 1 num-primes num-expected)
;;                 after handing out numbers and bounds; the transfer-primes handler
;;                 (core.clj:118-134) is not installed.
;;   client-start: replace (s/gen-table ...) / (s/sieve-e my-num false ...)
;;                 (core.clj:192,196) by (dse/run-machine! my-num n num-comps), with n and
;;                 num-comps sent by the lead instead of the bounds.
;;   -main:        parse N with Long/parseLong instead of Integer. (core.clj:210) to
;;                 reach N >= 2^31.
