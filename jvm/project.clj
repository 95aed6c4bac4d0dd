;; The JVM side of the drop-in: the reference's project (project.clj at its
;; root) plus JNA and this namespace. libdse.so must be on jna.library.path.
(defproject mail-sieve-e-dse "0.1.0"
  :description "mail-sieve-e's hot path on MI355X through libdse.so (JNA)"
  :dependencies [[org.clojure/clojure "1.6.0"]
                 [net.java.dev.jna/jna "5.14.0"]]
  :source-paths ["src"]
  :jvm-opts ["-Djna.library.path=../distributed-sieve-e_amd/mail_sieve_e"])
