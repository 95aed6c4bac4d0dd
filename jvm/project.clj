;; The JVM side of the drop-in: the reference's dependencies plus JNA, this
;; namespace (src/mail_sieve_e/dse.clj) next to the reference's core.clj with
;; its :require swapped to mail-sieve-e.dse. libdse.so must be on
;; jna.library.path.
(defproject mail-sieve-e-dse "0.1.0"
  :description "mail-sieve-e's hot path on MI355X through libdse.so (JNA)"
  :dependencies [[org.clojure/clojure "1.6.0"]
                 [org.clojure/core.async "0.1.346.0-17112a-alpha"]  ; the reference's, for core.clj
                 [net.java.dev.jna/jna "5.14.0"]]
  :source-paths ["src"]
  :jvm-opts ["-Djna.library.path=../distributed-sieve-e_amd/mail_sieve_e"])
